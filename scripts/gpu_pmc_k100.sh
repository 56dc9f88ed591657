#!/bin/bash
# rocprofv3 counter passes over the fp64 K=100 shard (config-5 per-GPU slice): HBM/L2 traffic of the
# E-step buckets (FETCH_SIZE, TCC hit/miss) -- one counter group per run, default .db output.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc100
i=0
for group in "FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc100/p$i
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $group -d gpurun_out/pmc100/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --converge 0 --e2e 0 --topics 100 --events 12500000 > gpurun_out/pmc100/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc100/p$i.log; exit 1; }
  db=$(find gpurun_out/pmc100/p$i -name "*.db" | head -1)
  python3 scripts/pmc_summary.py "$db" --match "oni::" --md gpurun_out/pmc100/p$i.md || exit 1
  rm -f "$db"
  echo "pass $i ok"
done
