# Full GPU tests after the bucket changes, then every BASELINE config on one GPU (fp64 engine).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/m_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -4 gpurun_out/m_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/bench_configs.sh
