set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
df -h /tmp | tail -1; free -g | head -2
timeout -k 10 1100 python -u scripts/config5.py --events 100000000 --days 30 --topics 100 --out gpurun_out/c5_100m.json > gpurun_out/c5_100m.log 2>&1 || { echo "config5 rc=$?"; tail -5 gpurun_out/c5_100m.log; exit 1; }
tail -1 gpurun_out/c5_100m.log; df -h /tmp | tail -1
