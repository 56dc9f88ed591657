# table-driven log also in gs_wteam / gs_wsteam (K <= 32): gs64 tests, headline bench, K = 20 bucket times
mkdir -p gpurun_out/r5ad
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5ad/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5ad/bench_k20.json 2> gpurun_out/r5ad/bench_k20.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --e2e 0 --e2e-cold 0 > gpurun_out/r5ad/bench_k20b.json 2> gpurun_out/r5ad/bench_k20b.err && \
timeout -k 10 300 python -u scripts/bench_gs64.py --reps 5 --phases > gpurun_out/r5ad/buckets_k20.log 2>&1
