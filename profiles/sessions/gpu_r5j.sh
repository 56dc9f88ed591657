# constant-offset row loads in the team / split kernels: oracle tests; K = 100 shard; config-5 100 M iteration
mkdir -p gpurun_out/r5j
true && \
true && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5j/bench_k100_12m.json 2> gpurun_out/r5j/bench_k100_12m.err && \
timeout -k 10 900 python -u bench.py --topics 100 --events 100000000 --steps 3 --warmup 1 --converge 0 > gpurun_out/r5j/bench_k100_100m.json 2> gpurun_out/r5j/bench_k100_100m.err
