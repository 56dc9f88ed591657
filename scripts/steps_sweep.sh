#!/bin/bash
# Timed-window sensitivity of the headline bench on one box (steps / warmup / batch).
set -o pipefail
mkdir -p gpurun_out/steps
for args in "--steps 20 --warmup 3" "--steps 30 --warmup 3" "--steps 20 --warmup 10" "--steps 60 --warmup 3" "--steps 20 --warmup 3" "--steps 20 --warmup 3 --batch 10"; do
  n=$(echo "$args" | tr ' -' '__')
  timeout -k 10 200 python bench.py $args --converge 0 --e2e 0 > gpurun_out/steps/$n.log 2>&1 || { echo "fail $args"; exit 1; }
  echo "$args $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/steps/$n.log)"
done
