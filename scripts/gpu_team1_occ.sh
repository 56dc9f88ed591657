# K>32 one-wave team occupancy variants (ONI_TEAM1_WAVES = 1 / 3 / 4): oracle tests, then bucket timing
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${TAG:-r2s4d}
for tw in 3 4; do
  ONI_TEAM1_WAVES=$tw timeout -k 10 200 python -u -m pytest tests/test_gs64.py -x -q --timeout 120 --timeout-method thread -k "estep_matches_oracle or em_run" > gpurun_out/${tag}_tw${tw}_test.log 2>&1 || { echo "tests tw=$tw failed"; tail -5 gpurun_out/${tag}_tw${tw}_test.log; exit 1; }
done
for tw in 1 3 4; do
  ONI_TEAM1_WAVES=$tw timeout -k 10 300 python -u scripts/bench_gs64.py --events 12500000 --topics 100 --warm-em 3 --reps 3 > gpurun_out/${tag}_k100_tw${tw}.json 2> gpurun_out/${tag}_k100_tw${tw}.err || { echo "bench tw=$tw failed"; tail -3 gpurun_out/${tag}_k100_tw${tw}.err; exit 1; }
done
echo done
