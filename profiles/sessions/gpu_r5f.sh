# K = 100 config-5 shard: per-bucket times and phase timers at U = 32 and U = 1024
mkdir -p gpurun_out/r5f
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --phases > gpurun_out/r5f/k100_u32.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 --phases > gpurun_out/r5f/k100_u1024.log 2>&1
