# re-entry check of HEAD on a fresh box: all GPU tests, smoke, default bench, cold ml_ops breakdown
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6ac
bash scripts/gpu.sh tests smoke bench cold || exit $?
