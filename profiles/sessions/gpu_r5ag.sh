# table log in also gs_team at KS > 32: gs64 tests, headline, K = 100 shard, buckets
mkdir -p gpurun_out/r5ag
timeout -k 10 500 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r5ag/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5ag/bench_k20.json 2> gpurun_out/r5ag/bench_k20.err && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --steps 10 --warmup 3 --converge 0 > gpurun_out/r5ag/bench_k100.json 2> gpurun_out/r5ag/bench_k100.err && \
timeout -k 10 300 python -u scripts/bench_gs64.py --events 12500000 --topics 100 --reps 5 > gpurun_out/r5ag/buckets_k100.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --reps 5 > gpurun_out/r5ag/buckets_k20.log 2>&1 && \
timeout -k 10 500 python -u bench.py --topics 100 --events 100000000 --steps 5 --warmup 2 --converge 0 > gpurun_out/r5ag/bench_k100_100m.json 2> gpurun_out/r5ag/bench_k100_100m.err
