mkdir -p gpurun_out/r5n
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 > gpurun_out/r5n/k100_u1024.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --only team8 --first 1 --phases > gpurun_out/r5n/k20_longest_phases.log 2>&1
