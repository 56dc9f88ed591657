#!/bin/bash
# rocprofv3 kernel trace of a short bench run + summary + E-step timeline.
#   PROF_NAME=k100 bash scripts/gpu_prof.sh --topics 100 --events 12500000
set -o pipefail
name=${PROF_NAME:-prof}
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m oni_ml_amd._build > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
rm -rf gpurun_out/$name
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$name -o run -- python3 bench.py --steps 5 --warmup 2 --converge 0 --e2e 0 "$@" > gpurun_out/$name.log 2>&1 || { tail -20 gpurun_out/$name.log; exit 1; }
python scripts/prof_summary.py gpurun_out/$name/run_results.db --md gpurun_out/${name}_summary.md > /dev/null
python scripts/timeline.py gpurun_out/$name/run_results.db --last-ms ${TIMELINE_MS:-1.5} > gpurun_out/${name}_timeline.txt
tail -3 gpurun_out/$name.log | grep metric | cut -c1-300
head -25 gpurun_out/${name}_summary.md
cat gpurun_out/${name}_timeline.txt
