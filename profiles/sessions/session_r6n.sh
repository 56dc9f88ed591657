set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gs64.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gs64.log 2>&1; rc=$?; tail -2 $O/pytest_gs64.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gs64.py --events 12500000 --topics 100 > $O/buckets_12m.log 2>&1 || exit 1
grep '^{' $O/buckets_12m.log | cut -c1-200
timeout -k 10 300 python -u scripts/lda_stage_ab.py --variants default,sync_pre --reps 3 --json $O/lda_stage_ab.json > $O/lda_stage_ab.log 2>&1 || exit 1
tail -2 $O/lda_stage_ab.log
timeout -k 10 600 python -u scripts/bench_gs64.py --events 100000000 --topics 100 > $O/buckets_100m.log 2>&1 || exit 1
grep '^{' $O/buckets_100m.log | cut -c1-200
