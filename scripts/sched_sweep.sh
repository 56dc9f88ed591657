#!/bin/bash
# E-step stream-schedule sweep (ONI_ESTEP_SCHED = side1 | side2 | side3 | main), headline bench.
set -o pipefail
mkdir -p gpurun_out/sched
i=0
for spec in ${SCHEDS:-"default"}; do
  i=$((i+1))
  if [ "$spec" = default ]; then unset ONI_ESTEP_SCHED; else export ONI_ESTEP_SCHED="$spec"; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --e2e 0 --converge 0 > gpurun_out/sched/$i.log 2>&1 || { echo "fail $spec"; tail -5 gpurun_out/sched/$i.log; exit 1; }
  echo "$spec $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sched/$i.log)"
done
