# final tree: all GPU tests, smoke, default bench, rocprof of the headline
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6as
bash scripts/gpu.sh tests smoke bench prof || exit $?
