# round-6 final-tree record: GPU tests, smoke, default bench, rocprof of the headline, K = 100 shard and 100 M events
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6u
bash scripts/gpu.sh tests smoke bench prof || exit $?
O=gpurun_out/r6u
timeout -k 10 400 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --e2e 0 --e2e-cold 0 > $O/bench_k100_12m.log 2>&1 || exit 1
grep '^{' $O/bench_k100_12m.log | tail -1 > $O/bench_k100_12m.json; cut -c1-400 $O/bench_k100_12m.json
timeout -k 10 600 python -u bench.py --topics 100 --events 100000000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0 > $O/bench_k100_100m.log 2>&1 || exit 1
grep '^{' $O/bench_k100_100m.log | tail -1 > $O/bench_k100_100m.json; cut -c1-400 $O/bench_k100_100m.json
