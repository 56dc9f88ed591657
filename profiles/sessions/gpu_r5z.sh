# per-stream suff-stats passes at KS > 32: gs64 tests; K = 100 shard and 100 M-event benches; 100 M timeline
mkdir -p gpurun_out/r5z
timeout -k 10 300 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread -k "suff or oracle" > gpurun_out/r5z/pytest_suff.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5z/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5z/bench_k100.json 2> gpurun_out/r5z/bench_k100.err && \
timeout -k 10 500 python -u bench.py --topics 100 --events 100000000 --steps 5 --warmup 2 --converge 0 > gpurun_out/r5z/bench_k100_100m.json 2> gpurun_out/r5z/bench_k100_100m.err && \
TAG=r5z_100m KEEP_GOING=0 PROF_ARGS="--topics 100 --events 100000000 --steps 3 --warmup 1 --converge 0 --e2e 0 --e2e-cold 0" TIMELINE_MS=200 bash scripts/gpu.sh prof > gpurun_out/r5z/prof.log 2>&1
