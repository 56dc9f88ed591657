#!/bin/bash
# GPU-box check: tests, the default bench, and a rocprofv3 kernel profile of the bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m oni_ml_amd._build > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" ; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -3 gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --converge 0 --e2e 0 > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof/run_results.db --md gpurun_out/prof_summary.md > /dev/null
echo done
