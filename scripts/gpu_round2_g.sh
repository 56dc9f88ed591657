set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ONI_THREADS=16
timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > gpurun_out/t_gpu_all.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/t_gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for tol in 1e-5 1e-6 1e-7; do
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --converge 0 --e2e 1 --e2e-tol $tol > gpurun_out/e2e_$tol.log 2>&1 || exit $?
  grep '^{' gpurun_out/e2e_$tol.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tol', d.get('e2e_flagged'), d.get('e2e_wall_s'), d.get('e2e_stage_s'))"
done
