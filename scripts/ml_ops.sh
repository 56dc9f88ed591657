#!/bin/bash
# Drop-in for the reference ml_ops.sh (YYYYMMDD TYPE [TOL]); extra flags pass through.
# GPUs: ONI_GPUS=N runs one process per GPU under torchrun (RCCL over xGMI).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="${HERE}${PYTHONPATH:+:${PYTHONPATH}}"
# malloc'd memory on transparent huge pages (glibc >= 2.35; read at process start, hence here): a cold flow
# day 1.748 -> 1.613 s spawn -> exit, median of 4 (fewer page faults in `import torch` and the pipeline,
# profiles/r6ai_cold_malloc.md)
export GLIBC_TUNABLES="glibc.malloc.hugetlb=1${GLIBC_TUNABLES:+:${GLIBC_TUNABLES}}"
N=${ONI_GPUS:-1}
if [[ "${N}" -gt 1 ]]; then
  exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "${N}" --master-addr 127.0.0.1 \
       --master-port "${MASTER_PORT:-29531}" -m oni_ml_amd ml_ops "$@" --gpus "${N}"
fi
exec python -m oni_ml_amd ml_ops "$@"
