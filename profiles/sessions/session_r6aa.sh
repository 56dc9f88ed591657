# team4 on c.phi-row tables at 3 waves per SIMD (K > 32) and the split's per-KS segment target: oracle tests,
# then K = 50, the K = 100 shard and 100 M events
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6aa; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gs64.py tests/test_lda_hip.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --topics 50 --steps 20 --warmup 3 --e2e 0 --e2e-cold 0 > $O/bench_k50.log 2>&1 || exit 1
grep '^{' $O/bench_k50.log | tail -1 > $O/bench_k50.json; cut -c1-300 $O/bench_k50.json
timeout -k 10 400 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --e2e 0 --e2e-cold 0 > $O/bench_k100_12m.log 2>&1 || exit 1
grep '^{' $O/bench_k100_12m.log | tail -1 > $O/bench_k100_12m.json; cut -c1-300 $O/bench_k100_12m.json
timeout -k 10 600 python -u bench.py --topics 100 --events 100000000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0 > $O/bench_k100_100m.log 2>&1 || exit 1
grep '^{' $O/bench_k100_100m.log | tail -1 > $O/bench_k100_100m.json; cut -c1-300 $O/bench_k100_100m.json
