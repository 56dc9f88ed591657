# late suff-stats pass = the last-finishing bucket (team8 at K > 32): gs64 tests; K = 100 shard bench + timeline; headline bench
mkdir -p gpurun_out/r5t
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5t/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5t/bench_k100.json 2> gpurun_out/r5t/bench_k100.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5t/bench_k20.json 2> gpurun_out/r5t/bench_k20.err && \
TAG=r5t_k100 KEEP_GOING=0 PROF_ARGS="--topics 100 --events 12500000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0" TIMELINE_MS=40 bash scripts/gpu.sh prof > gpurun_out/r5t/prof.log 2>&1
