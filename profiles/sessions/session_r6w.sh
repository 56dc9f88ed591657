# LAG saves through device handoffs + log-beta kernel + capture prelaunch: GPU tests of the touched paths, then
# the lda-stage A/B, the to-convergence A/B and the default bench (cold ml_ops child)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lda_hip.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/lda_stage_ab.py --variants default,sync_pre --reps 3 --json $O/lda_stage_ab.json > $O/lda_stage_ab.log 2>&1 || exit 1
tail -2 $O/lda_stage_ab.log | cut -c1-600
timeout -k 10 300 python -u scripts/converge_ab.py --reps 7 > $O/converge_ab.log 2>&1 || exit 1
grep '^{' $O/converge_ab.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log | tail -1 > $O/bench.json; cut -c1-300 $O/bench.json
