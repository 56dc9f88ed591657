# final-tree evidence: rocprofv3 kernel traces (headline K = 20, K = 100 shard) and the 100 M-event K = 100 iteration
export KEEP_GOING=0
TAG=r5q_k20 bash scripts/gpu.sh prof && \
TAG=r5q_k100 PROF_ARGS="--topics 100 --events 12500000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0" TIMELINE_MS=40 bash scripts/gpu.sh prof && \
timeout -k 10 900 python -u bench.py --topics 100 --events 100000000 --steps 3 --warmup 1 --converge 0 > gpurun_out/r5q_k100/bench_100m.json 2> gpurun_out/r5q_k100/bench_100m.err
