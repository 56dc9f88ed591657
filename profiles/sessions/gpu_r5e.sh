export TAG=r5e KEEP_GOING=1
bash scripts/gpu.sh tests && \
timeout -k 10 240 python -u scripts/bench_gs64.py --xsplit 1 --xsplit-g 32 --only split --phases > gpurun_out/r5e/xs32.log 2>&1 && \
timeout -k 10 240 python -u scripts/bench_gs64.py --xsplit 1 --only split --phases > gpurun_out/r5e/xs1.log 2>&1 && \
timeout -k 10 240 python -u scripts/bench_gs64.py --xsplit 2 > gpurun_out/r5e/xs2_all.log 2>&1 && \
timeout -k 10 240 python -u scripts/bench_gs64.py > gpurun_out/r5e/base_all.log 2>&1 && \
BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu.sh bench
