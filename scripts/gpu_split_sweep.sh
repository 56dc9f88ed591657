# fp64 K=100 split-document sweep: gs64 tests, per-bucket timing under split settings, K=100 bench
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${TAG:-r2s4b}
timeout -k 10 300 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_gs64_test.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/${tag}_gs64_test.log | head; exit 1; }
for cfg in ${CFGS:-16384:16 8192:16}; do
  set -- ${cfg/:/ }
  ONI_GS_SPLIT_MIN=$1 ONI_GS_SPLIT_G=$2 timeout -k 10 300 python -u scripts/bench_gs64.py --events 12500000 --topics 100 --warm-em 3 --reps 3 > gpurun_out/${tag}_k100_min$1_g$2.json 2> gpurun_out/${tag}_k100_min$1_g$2.err || { echo "bench $cfg failed"; tail -3 gpurun_out/${tag}_k100_min$1_g$2.err; exit 1; }
done
timeout -k 10 400 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --e2e 0 > gpurun_out/${tag}_bench_k100.json 2> gpurun_out/${tag}_bench_k100.err || { echo "bench.py failed"; tail -3 gpurun_out/${tag}_bench_k100.err; exit 1; }
echo done
