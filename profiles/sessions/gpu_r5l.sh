# cold DNS after moving dns_pre's host features onto the prefetch thread
mkdir -p gpurun_out/r5l
timeout -k 10 500 python -u scripts/cold_start.py --source dns --events 2000000 --reps 3 --variants "default;ONI_PREFETCH=0" --md gpurun_out/r5l/cold_dns.md --json gpurun_out/r5l/cold_dns.json --prof-out gpurun_out/r5l/dns.prof > gpurun_out/r5l/cold_dns.log 2>&1
