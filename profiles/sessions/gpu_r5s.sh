# paired loads at KS 52/64 and in gs_smallw: all gs64 oracle tests; K = 100 shard; K = 50 (config 3); PMC at K = 100
mkdir -p gpurun_out/r5s
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5s/pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 > gpurun_out/r5s/k100_u32.log 2>&1 && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5s/bench_k100.json 2> gpurun_out/r5s/bench_k100.err && \
timeout -k 10 300 python -u bench.py --topics 50 --steps 20 --warmup 5 --converge 0 > gpurun_out/r5s/bench_k50.json 2> gpurun_out/r5s/bench_k50.err && \
timeout -k 10 300 python -u bench.py --topics 50 --gs-updates 64 --steps 20 --warmup 5 --converge 0 > gpurun_out/r5s/bench_k50_u64.json 2> gpurun_out/r5s/bench_k50_u64.err && \
TAG=r5s KEEP_GOING=0 PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;TCC_HIT_sum TCC_MISS_sum" \
PMC_MATCH="gs_" PMC_ARGS="--topics 100 --events 12500000 --steps 3 --warmup 1 --converge 0" bash scripts/gpu.sh pmc > gpurun_out/r5s/pmc.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 > gpurun_out/r5s/k100_u1024.log 2>&1
