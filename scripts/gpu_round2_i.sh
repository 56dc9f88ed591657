set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/t_gpu_all2.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -4 gpurun_out/t_gpu_all2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/config5.py --events 10000000 --days 10 --topics 100 --em-iters 2 --out gpurun_out/c5_10m.json > gpurun_out/c5_10m.log 2>&1 || { echo "config5 rc=$?"; tail -5 gpurun_out/c5_10m.log; exit 1; }
tail -1 gpurun_out/c5_10m.log
