# full GPU test suite, headline bench, precision/schedule parity on the headline corpus
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ONI_THREADS=16
timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > gpurun_out/t_gpu_all.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/t_gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench_r2.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_r2.log | cut -c1-1500
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -u scripts/precision_parity.py --json gpurun_out/r2_precision_parity.json --md gpurun_out/r2_precision_parity.md > gpurun_out/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; cat gpurun_out/r2_precision_parity.md
