# round-6 records of the other BASELINE configs on one GPU, a cold DNS ml_ops, and the config-5 month through
# ml_ops on one GPU
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6x COLD_ARGS="--source dns --events 2000000 --reps 2 --variants default"
bash scripts/gpu.sh configs cold || exit $?
O=$GRAFT_REPO_ROOT/gpurun_out/r6x
timeout -k 10 800 python -u scripts/pipeline_ranks.py --events 100000000 --days 30 --topics 100 --compat fixed \
  --tol 2.93e-8 --lag 0 --ranks 1 --threads 16 --timeout 600 --json $O/c5_one_gpu.json --md $O/c5_one_gpu.md \
  > $O/c5_one_gpu.log 2>&1; rc=$?
cat $O/c5_one_gpu.md | head -14; exit $rc
