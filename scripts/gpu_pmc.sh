#!/bin/bash
# rocprofv3 hardware-counter passes (one counter group per run) over a short bench run.
#   PMC_NAME=k20 bash scripts/gpu_pmc.sh [bench args]
set -o pipefail
name=${PMC_NAME:-pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for group in "FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf gpurun_out/${name}_p$i
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $group -d gpurun_out/${name}_p$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --converge 0 --e2e 0 "$@" > gpurun_out/${name}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${name}_p$i.log; exit 1; }
  echo "pass $i ok"
done
