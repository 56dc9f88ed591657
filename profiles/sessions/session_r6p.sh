# team4 prefetch depth A/B (TEAM4_RMAX 3 = this tree's build, 1 = round 5, 2) on the K = 100 shard; oracle tests first
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; cd "$R"
O=$R/gpurun_out/r6p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gs64.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gs64.log 2>&1; rc=$?; tail -2 $O/pytest_gs64.log; [ $rc -eq 0 ] || exit $rc
for v in r3 r1 r2 r3b; do
  rm -rf /tmp/v_$v; cp -r "$R" /tmp/v_$v
  case $v in r1|r2) cp abvar/$v/_onihip*.so /tmp/v_$v/oni_ml_amd/_lib/ ;; esac
  (cd /tmp/v_$v && timeout -k 10 300 python -u scripts/bench_gs64.py --events 12500000 --topics 100 > $O/buckets_12m_$v.log 2>&1) || exit 1
  echo "== $v"; grep '^{' $O/buckets_12m_$v.log | cut -c1-160
  rm -rf /tmp/v_$v
done
timeout -k 10 600 python -u scripts/bench_gs64.py --events 100000000 --topics 100 > $O/buckets_100m.log 2>&1 || exit 1
grep '^{' $O/buckets_100m.log | cut -c1-200
