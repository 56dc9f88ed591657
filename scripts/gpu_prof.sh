#!/bin/bash
# rocprofv3 kernel trace of a short bench run + summary + E-step timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m oni_ml_amd._build > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --converge 0 --e2e 0 "$@" > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof/run_results.db --md gpurun_out/prof_summary.md > /dev/null
python scripts/timeline.py gpurun_out/prof/run_results.db --last-ms 1.5 > gpurun_out/timeline.txt
tail -3 gpurun_out/prof.log | grep metric | cut -c1-300
head -25 gpurun_out/prof_summary.md
cat gpurun_out/timeline.txt
