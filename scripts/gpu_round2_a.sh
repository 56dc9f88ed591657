set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gs64.py > gpurun_out/t_gs64.log 2>&1
rc=$?
echo "gs64 rc=$rc"
grep -E "PASS|FAIL" gpurun_out/t_gs64.log
exit $rc
