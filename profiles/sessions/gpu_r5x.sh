# K > 32 bucket-edge sweep: team8 vs team4 for the 2 k+ word documents, 12.5 M shard and 100 M events
mkdir -p gpurun_out/r5x
timeout -k 10 500 python -u scripts/edges_sweep.py --events 12500000 --variants default t4all t8_4k t8_8k > gpurun_out/r5x/edges.log 2>&1 && \
timeout -k 10 600 python -u scripts/edges_sweep.py --events 100000000 --variants t4all t8_4k t8_8k >> gpurun_out/r5x/edges.log 2>&1
