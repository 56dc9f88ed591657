mkdir -p gpurun_out/r5n
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 > gpurun_out/r5n/k100_u1024.log 2>&1
