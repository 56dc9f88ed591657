#!/bin/bash
# Drop-in for the reference ml_ops.sh (YYYYMMDD TYPE [TOL]); extra flags pass through.
# GPUs: ONI_GPUS=N runs one process per GPU under torchrun (RCCL over xGMI).
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
export PYTHONPATH="${HERE}${PYTHONPATH:+:${PYTHONPATH}}"
N=${ONI_GPUS:-1}
if [[ "${N}" -gt 1 ]]; then
  exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "${N}" --master-addr 127.0.0.1 \
       --master-port "${MASTER_PORT:-29531}" -m oni_ml_amd ml_ops "$@" --gpus "${N}"
fi
exec python -m oni_ml_amd ml_ops "$@"
