# U = 1024 at K = 100: split segment sizes; K = 50 config-3 parity schedule (U = 64) and default
mkdir -p gpurun_out/r5o
for spec in "2048,words=16" "2048,words=32" "8000,words=16"; do
  echo "=== spec '$spec'" >> gpurun_out/r5o/u1024_split.log
  ONI_GS_SPLIT_MIN="$spec" timeout -k 10 200 python -u scripts/bench_gs64.py --topics 100 --events 12500000 --gs-updates 1024 >> gpurun_out/r5o/u1024_split.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --topics 50 --steps 20 --warmup 5 --converge 0 > gpurun_out/r5o/k50_u32.json 2> gpurun_out/r5o/k50_u32.err && \
timeout -k 10 300 python -u bench.py --topics 50 --gs-updates 64 --steps 20 --warmup 5 --converge 0 > gpurun_out/r5o/k50_u64.json 2> gpurun_out/r5o/k50_u64.err && \
timeout -k 10 300 python -u bench.py --topics 100 --events 12500000 --gs-updates 1024 --steps 5 --warmup 2 --converge 0 > gpurun_out/r5o/k100_u1024.json 2> gpurun_out/r5o/k100_u1024.err
