# final-tree record after the team4 / split-plan changes: all GPU tests, smoke, default bench, K = 50
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6ab
bash scripts/gpu.sh tests smoke bench || exit $?
O=gpurun_out/r6ab
timeout -k 10 900 bash scripts/ab_env.sh 2 "ONI_GS_SPLIT_MIN=" "ONI_GS_SPLIT_MIN=2048,words=96" -- --topics 50 --steps 20 --warmup 5 > $O/ab_k50.log 2>&1 || exit 1
cat $O/ab_k50.log
