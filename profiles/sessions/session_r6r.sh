# 8 ranks sharing one GPU, a quarter of config 5 (25 M events, K = 100): where flow_pre's time goes
# (ONI_THREADS=16 vs the per-rank budget), every rank under cProfile
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6r; mkdir -p $O
timeout -k 10 1000 python -u scripts/pipeline_ranks.py --events 25000000 --days 8 --topics 100 --compat fixed \
  --tol 2.93e-8 --lag 0 --ranks 8 --threads 0 --variants ';ONI_THREADS=16' --timeout 420 \
  --env "ONI_PROFILE=cprofile:$O/prof_{rank}.out" --json $O/ranks.json --md $O/ranks.md > $O/ranks.log 2>&1; rc=$?
for r in 0 1; do python -c "import pstats,sys; pstats.Stats('$O/prof_$r.out').sort_stats('tottime').print_stats(25)" > $O/prof_$r.txt 2>&1; done
tail -3 $O/ranks.log | cut -c1-300; head -40 $O/prof_1.txt; exit $rc
