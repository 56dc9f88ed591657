# after the table log: 100 M events, K = 50 flow day (U = 32 and 64), K = 100 shard timeline
mkdir -p gpurun_out/r5af
timeout -k 10 500 python -u bench.py --topics 100 --events 100000000 --steps 5 --warmup 2 --converge 0 > gpurun_out/r5af/bench_k100_100m.json 2> gpurun_out/r5af/bench_k100_100m.err && \
timeout -k 10 300 python -u bench.py --topics 50 --steps 20 --warmup 5 --converge 0 --e2e 0 --e2e-cold 0 > gpurun_out/r5af/bench_k50.json 2> gpurun_out/r5af/bench_k50.err && \
timeout -k 10 300 python -u bench.py --topics 50 --gs-updates 64 --steps 20 --warmup 5 --converge 0 --e2e 0 --e2e-cold 0 > gpurun_out/r5af/bench_k50_u64.json 2> gpurun_out/r5af/bench_k50_u64.err && \
TAG=r5af_k100 KEEP_GOING=0 PROF_ARGS="--topics 100 --events 12500000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0" TIMELINE_MS=40 bash scripts/gpu.sh prof > gpurun_out/r5af/prof.log 2>&1
