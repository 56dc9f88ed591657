# 8 ranks sharing one GPU (25 M events, K = 100), one hardware queue per rank (8 in all instead of 32):
# the host-resource variants without HW-queue oversubscription
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6t; mkdir -p $O
timeout -k 10 1000 python -u scripts/pipeline_ranks.py --events 25000000 --days 8 --topics 100 --compat fixed \
  --tol 2.93e-8 --lag 0 --ranks 8 --threads 0 --timeout 450 --env GPU_MAX_HW_QUEUES=1 \
  --variants "ONI_PROFILE=cprofile:$O/pa_{rank}.out;ONI_THREADS=16,ONI_PROFILE=cprofile:$O/pb_{rank}.out" \
  --json $O/ranks.json --md $O/ranks.md > $O/ranks.log 2>&1; rc=$?
for v in pa pb; do for r in 0 1; do python -c "import pstats; pstats.Stats('$O/${v}_$r.out').sort_stats('tottime').print_stats(15)" > $O/${v}_$r.txt 2>&1; done; done
cat $O/ranks.md | grep -v "^| [2-7] "; head -25 $O/pa_1.txt | tail -14; exit $rc
