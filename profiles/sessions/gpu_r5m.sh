# gs_chain (per-word chains at K > 32, U > 32): oracle tests; K = 100 shard at U = 1024; cold DNS with host cuts
mkdir -p gpurun_out/r5m
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5m/pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 > gpurun_out/r5m/k100_u1024.log 2>&1 && \
timeout -k 10 500 python -u scripts/cold_start.py --source dns --events 2000000 --reps 3 --variants "default" --md gpurun_out/r5m/cold_dns.md --json gpurun_out/r5m/cold_dns.json > gpurun_out/r5m/cold_dns.log 2>&1
