#!/bin/bash
# GPU-box check: tests, a short bench, and a rocprofv3 kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" ; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --corpus planted --steps 5 --warmup 2 --converge 0 > gpurun_out/bench_planted.log 2>&1 || exit 1
cat gpurun_out/bench_planted.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --corpus planted --steps 3 --warmup 1 --converge 0 > gpurun_out/prof.log 2>&1 || exit 1
find gpurun_out/prof -name '*stats*' | head
