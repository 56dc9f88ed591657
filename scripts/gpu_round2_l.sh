# After the longest-document kernel work: all GPU tests, default bench, fp64 kernel profile + phases.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof64l
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/l_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -4 gpurun_out/l_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/l_bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/l_bench.log; exit 1; }
tail -1 gpurun_out/l_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64l -o run -- python3 bench.py --steps 10 --warmup 3 --converge 0 --e2e 0 > gpurun_out/prof64l/bench.log 2>&1 || { echo "prof rc=$?"; tail -20 gpurun_out/prof64l/bench.log; exit 1; }
db=$(find gpurun_out/prof64l -name "*.db" | head -1)
python scripts/prof_summary.py "$db" --top 30 --md gpurun_out/prof64l/summary.md > /dev/null
python scripts/timeline.py "$db" --last-ms 6 > gpurun_out/prof64l/timeline.txt
rm -f "$db"
head -12 gpurun_out/prof64l/summary.md
timeout -k 10 300 python -u scripts/bench_gs64.py --phases > gpurun_out/l_phases.log 2>&1 || { echo "gs64 rc=$?"; tail -20 gpurun_out/l_phases.log; exit 1; }
grep '^{' gpurun_out/l_phases.log | cut -c1-300
