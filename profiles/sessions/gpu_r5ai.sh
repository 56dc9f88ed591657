# full GPU test suite, smoke, headline bench (default arguments), K = 100 shard bench
mkdir -p gpurun_out/r5ai
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5ai/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5ai/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5ai/bench_default.json 2> gpurun_out/r5ai/bench_default.err && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5ai/bench_k100.json 2> gpurun_out/r5ai/bench_k100.err
