set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./scripts/micro/fp64_latency > gpurun_out/fp64_latency.txt 2>&1; echo "micro rc=$?"; cat gpurun_out/fp64_latency.txt
mkdir -p gpurun_out/prof64; rm -rf gpurun_out/prof64/*
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run -- python3 bench.py --steps 10 --warmup 3 --converge 0 --e2e 0 > gpurun_out/prof64/bench.log 2>&1
echo "prof rc=$?"
grep '^{' gpurun_out/prof64/bench.log | cut -c1-300
db=$(find gpurun_out/prof64 -name "*.db" | head -1)
python scripts/prof_summary.py "$db" --top 6
