# tiny keeps fexp at KS <= 32: gs64 tests, headline bench twice, K = 100 shard
mkdir -p gpurun_out/r5ar
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5ar/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5ar/bench_default.json 2> gpurun_out/r5ar/bench_default.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e2e 0 --e2e-cold 0 > gpurun_out/r5ar/bench_k20b.json 2> gpurun_out/r5ar/bench_k20b.err && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5ar/bench_k100.json 2> gpurun_out/r5ar/bench_k100.err
