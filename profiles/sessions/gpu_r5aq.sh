# final-tree record: full GPU suite, smoke, default bench, headline rocprof summary + timeline, K = 100 shard
mkdir -p gpurun_out/r5aq
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r5aq/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5aq/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5aq/bench_default.json 2> gpurun_out/r5aq/bench_default.err && \
TAG=r5aq_k20 KEEP_GOING=0 TIMELINE_MS=6 bash scripts/gpu.sh prof > gpurun_out/r5aq/prof_k20.log 2>&1 && \
TAG=r5aq_k100 KEEP_GOING=0 PROF_ARGS="--topics 100 --events 12500000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0" TIMELINE_MS=40 bash scripts/gpu.sh prof > gpurun_out/r5aq/prof_k100.log 2>&1
