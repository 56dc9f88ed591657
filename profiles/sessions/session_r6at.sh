# final-tree BASELINE configs on one GPU (headline, K = 50, DNS K = 20, config-5 shard) and the 100 M-event month
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6at
mkdir -p $O
OUTDIR=$O bash scripts/bench_configs.sh || exit 1
timeout -k 10 600 python -u bench.py --topics 100 --events 100000000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0 > $O/bench_k100_100m.log 2>&1 || exit 1
grep '^{' $O/bench_k100_100m.log | tail -1 > $O/bench_k100_100m.json; cut -c1-300 $O/bench_k100_100m.json
