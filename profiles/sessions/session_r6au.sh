# the config-5 month (100 M events, K = 100) through ml_ops on one GPU on the final tree (sort-based group-bys
# at 200 M keys, the device ECDF kept above 4 M rows)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6au
mkdir -p $O
timeout -k 10 900 python -u scripts/pipeline_ranks.py --events 100000000 --days 30 --topics 100 --compat fixed \
  --tol 2.93e-8 --lag 0 --ranks 1 --threads 16 --timeout 700 --json $O/c5_one_gpu.json --md $O/c5_one_gpu.md \
  > $O/c5_one_gpu.log 2>&1; rc=$?
cat $O/c5_one_gpu.md | head -14; exit $rc
