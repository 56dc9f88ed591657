# rocprofv3 kernel traces of the round-5 tree: headline (K = 20) and the K = 100 config-5 shard
export KEEP_GOING=0
TAG=r5q_k20 bash scripts/gpu.sh prof && \
TAG=r5q_k100 PROF_ARGS="--topics 100 --events 12500000 --steps 5 --warmup 2 --converge 0 --e2e 0 --e2e-cold 0" TIMELINE_MS=40 bash scripts/gpu.sh prof
