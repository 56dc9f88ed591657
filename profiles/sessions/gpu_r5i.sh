# K = 100 shard, U = 32: split plan sweep (graph time is the number that matters)
mkdir -p gpurun_out/r5i
for spec in "" "2048,words=64" "2048,words=96" "2048,batches=2" "4096,words=64" "1500,words=96,batches=2"; do
  echo "=== spec '$spec'" >> gpurun_out/r5i/sweep.log
  ONI_GS_SPLIT_MIN="$spec" timeout -k 10 200 python -u scripts/bench_gs64.py --topics 100 --events 12500000 >> gpurun_out/r5i/sweep.log 2>&1 || exit 1
done
