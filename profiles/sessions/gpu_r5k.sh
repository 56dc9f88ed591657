# cold ml_ops processes after the round-5 pruning: DNS 2 M queries and flow 1 M events
mkdir -p gpurun_out/r5k
timeout -k 10 500 python -u scripts/cold_start.py --source dns --events 2000000 --reps 3 --variants "default" --md gpurun_out/r5k/cold_dns.md --json gpurun_out/r5k/cold_dns.json --prof-out gpurun_out/r5k/dns.prof > gpurun_out/r5k/cold_dns.log 2>&1 && \
timeout -k 10 500 python -u scripts/cold_start.py --source flow --events 1000000 --reps 3 --variants "default" --md gpurun_out/r5k/cold_flow.md --json gpurun_out/r5k/cold_flow.json --prof-out gpurun_out/r5k/flow.prof > gpurun_out/r5k/cold_flow.log 2>&1
