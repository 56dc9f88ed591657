# rocprofv3 kernel trace of the fp64 headline bench (10 timed EM iterations)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof64
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run -- python3 bench.py --steps 10 --warmup 3 --converge 0 --e2e 0 > gpurun_out/prof64/bench.log 2>&1
rc=$?
echo "prof rc=$rc"
ls -R gpurun_out/prof64 | head -20
db=$(find gpurun_out/prof64 -name "*.db" | head -1)
csv=$(find gpurun_out/prof64 -name "*kernel_trace.csv" | head -1)
if [ -n "$db" ]; then python scripts/prof_summary.py "$db" --top 25; python scripts/timeline.py "$db" --last-ms 4 > gpurun_out/prof64/timeline.txt; elif [ -n "$csv" ]; then python scripts/prof_summary.py "$csv" --top 25; fi
exit $rc
