# branch-free refreshes + gs_smallw at K > 32 + batched split exchange + split at U > 32 (scratch tables):
# oracle tests, K = 100 shard at U = 32 / 1024, headline
mkdir -p gpurun_out/r5h
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5h/pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --phases > gpurun_out/r5h/k100_u32.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 --phases > gpurun_out/r5h/k100_u1024.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py > gpurun_out/r5h/k20.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5h/bench.json 2> gpurun_out/r5h/bench.err
