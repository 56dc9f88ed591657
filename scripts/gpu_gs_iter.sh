# fp64 E-step iteration loop: gs64 GPU tests, per-bucket phases for kernel variants, bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/test_gs64.py > gpurun_out/it_gs64.log 2>&1
rc=$?; echo "gs64 tests rc=$rc"; tail -3 gpurun_out/it_gs64.log
if [ $rc -ne 0 ]; then exit $rc; fi
for cfg in ${CFGS:-"X=0"}; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python -u scripts/bench_gs64.py --phases ${GSARGS:-} > gpurun_out/it_phases.log 2>&1 || { echo "phases rc=$?"; tail -20 gpurun_out/it_phases.log; exit 1; }
  grep '^{' gpurun_out/it_phases.log | cut -c1-300
  env $cfg timeout -k 10 300 python -u bench.py --e2e 0 --converge 0 > gpurun_out/it_bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/it_bench.log; exit 1; }
  tail -1 gpurun_out/it_bench.log | grep -o '"ms_per_step": [0-9.]*'
done
