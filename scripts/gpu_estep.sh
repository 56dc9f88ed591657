#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -m oni_ml_amd._build > gpurun_out/build.log 2>&1 || { tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?"; tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 600 python scripts/bench_estep.py "$@" > gpurun_out/bench_estep.log 2>&1 || { tail -30 gpurun_out/bench_estep.log; exit 1; }
cat gpurun_out/bench_estep.log | python3 -c "
import json,sys
for l in sys.stdin:
    if not l.startswith('{'): continue
    d=json.loads(l)
    if 'rows' not in d: print(l.strip()); continue
    print('split_min', d['split_min'])
    for r in d['rows']: print('  ', r)
"
