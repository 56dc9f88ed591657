# fp64 buckets at K = 50 (1M-event day) and K = 100 (12.5M-event shard).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_gs64.py --phases --topics 50 > gpurun_out/w50.log 2>&1 || { echo "k50 rc=$?"; tail -20 gpurun_out/w50.log; exit 1; }
grep '^{' gpurun_out/w50.log | cut -c1-330
timeout -k 10 400 python -u scripts/bench_gs64.py --phases --topics 100 --events 12500000 --reps 3 > gpurun_out/w100.log 2>&1 || { echo "k100 rc=$?"; tail -20 gpurun_out/w100.log; exit 1; }
grep '^{' gpurun_out/w100.log | cut -c1-330
