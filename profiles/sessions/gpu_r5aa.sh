# refactored per-stream suff-stats plan: suff / oracle gs64 tests, K = 100 shard bench, headline bench
mkdir -p gpurun_out/r5aa
timeout -k 10 300 python -u -m pytest tests/test_gs64.py tests/test_suff_groups.py -x -v --timeout 120 --timeout-method thread -k "suff or oracle or group" > gpurun_out/r5aa/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5aa/bench_k100.json 2> gpurun_out/r5aa/bench_k100.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5aa/bench_k20.json 2> gpurun_out/r5aa/bench_k20.err
