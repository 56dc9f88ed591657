# paired-topic loads (KS > 64): oracle tests at K >= 50, K = 100 shard buckets with phases
mkdir -p gpurun_out/r5r
timeout -k 10 400 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread -k "100 or 128 or 50 or 64 or split" > gpurun_out/r5r/pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --phases > gpurun_out/r5r/k100_u32.log 2>&1 && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5r/bench_k100.json 2> gpurun_out/r5r/bench_k100.err && \
timeout -k 10 300 python -u scripts/engine_setup_profile.py --out gpurun_out/r5r/setup.txt > gpurun_out/r5r/setup.log 2>&1
