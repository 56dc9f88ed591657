# fp64 engine: numerics tests, per-bucket timing, PMC pass on the tiny-document kernel
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gs64.py > gpurun_out/t_gs64.log 2>&1
rc=$?; echo "gs64 rc=$rc"; tail -3 gpurun_out/t_gs64.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/bench_gs64.py > gpurun_out/bench_gs64.txt 2>&1; rc=$?; echo "buckets rc=$rc"; cat gpurun_out/bench_gs64.txt | grep "^{"
if [ $rc -ne 0 ]; then exit $rc; fi
rm -rf gpurun_out/pmc_tiny; mkdir -p gpurun_out/pmc_tiny
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD -d gpurun_out/pmc_tiny -o pmc -- python3 scripts/bench_gs64.py --only tiny --reps 2 > gpurun_out/pmc_tiny/log.txt 2>&1
echo "pmc rc=$?"
find gpurun_out/pmc_tiny -name "*counter_collection*" | head
