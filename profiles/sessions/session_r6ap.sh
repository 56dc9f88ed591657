# final-tree record after the cold-path work: all GPU tests, smoke, default bench, DNS cold ml_ops, K = 100 shard
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6ap
bash scripts/gpu.sh tests smoke bench || exit $?
O=gpurun_out/r6ap
timeout -k 10 600 python -u scripts/cold_start.py --source dns --events 2000000 --reps 2 --variants "default" --md $O/cold_dns.md --json $O/cold_dns.json > $O/cold_dns.log 2>&1 || exit 1
grep median $O/cold_dns.md
timeout -k 10 400 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --e2e 0 --e2e-cold 0 > $O/bench_k100_12m.log 2>&1 || exit 1
grep '^{' $O/bench_k100_12m.log | tail -1 > $O/bench_k100_12m.json; cut -c1-300 $O/bench_k100_12m.json
