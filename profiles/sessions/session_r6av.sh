# final tree after the O(n) run starts / segment ids: all GPU tests, smoke, bench, then the config-5 month on one GPU
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6av
bash scripts/gpu.sh tests smoke bench || exit $?
O=$GRAFT_REPO_ROOT/gpurun_out/r6av
timeout -k 10 900 python -u scripts/pipeline_ranks.py --events 100000000 --days 30 --topics 100 --compat fixed \
  --tol 2.93e-8 --lag 0 --ranks 1 --threads 16 --timeout 700 --json $O/c5_one_gpu.json --md $O/c5_one_gpu.md \
  > $O/c5_one_gpu.log 2>&1; rc=$?
cat $O/c5_one_gpu.md | head -10; exit $rc
