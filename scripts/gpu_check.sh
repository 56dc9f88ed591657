#!/bin/bash
# GPU tests (optionally a -k filter) + per-config bench lines.  Usage:
#   bash scripts/gpu_check.sh [pytest -k expr] -- [bench_configs args]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${PYTEST_K:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu.log
exit $rc
