# fp64 engine: numerics tests, then a kernel-trace profile of the headline bench
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof64
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gs64.py > gpurun_out/t_gs64.log 2>&1
rc=$?
echo "gs64 rc=$rc"; grep -cE "PASSED" gpurun_out/t_gs64.log; grep -E "FAILED" gpurun_out/t_gs64.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
rm -rf gpurun_out/prof64/*
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run -- python3 bench.py --steps 10 --warmup 3 --converge 1 --e2e 0 > gpurun_out/prof64/bench.log 2>&1
echo "prof rc=$?"
tail -c 1500 gpurun_out/prof64/bench.log
db=$(find gpurun_out/prof64 -name "*.db" | head -1)
python scripts/prof_summary.py "$db" --top 8
