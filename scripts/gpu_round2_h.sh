set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gs64.py > gpurun_out/t_gs64.log 2>&1
rc=$?; echo "gs64 rc=$rc"; tail -2 gpurun_out/t_gs64.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for nw in 4 8; do
  ONI_GS_BIG_NW=$nw timeout -k 10 300 python -u scripts/bench_gs64.py --phases --only team8 > gpurun_out/ph_$nw.txt 2>&1 || exit $?
  echo "NW=$nw"; grep "^{" gpurun_out/ph_$nw.txt
done
