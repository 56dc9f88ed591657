# gs_smallw (16 lanes per document at K > 32): oracle tests, then K = 100 shard buckets at U = 32 / 1024
mkdir -p gpurun_out/r5g
timeout -k 10 400 python -u -m pytest tests/test_gs64.py -x -v --timeout 120 --timeout-method thread -k "estep_matches_oracle or final_pass or large_u or cphi_windows or suff_split or em_run" > gpurun_out/r5g/pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 > gpurun_out/r5g/k100_u32.log 2>&1 && \
timeout -k 10 300 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 > gpurun_out/r5g/k100_u1024.log 2>&1
