# 100 M events at K = 100: bucket times alone (bench_gs64 --phases) and the rocprof timeline of the EM iteration
mkdir -p gpurun_out/r5y
timeout -k 10 500 python -u scripts/bench_gs64.py --events 100000000 --topics 100 --reps 3 --warm-em 2 --phases > gpurun_out/r5y/buckets_100m.log 2>&1 && \
TAG=r5y_100m KEEP_GOING=0 PROF_ARGS="--topics 100 --events 100000000 --steps 3 --warmup 1 --converge 0 --e2e 0 --e2e-cold 0" TIMELINE_MS=200 bash scripts/gpu.sh prof > gpurun_out/r5y/prof.log 2>&1
