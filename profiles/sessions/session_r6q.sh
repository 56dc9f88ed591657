# K = 100 bucket edges: the 16-lane kernel's upper edge (256 -> 128 / 512 / 1024); pinned-buffer first-use cost
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 120 python -u scripts/pinned_alloc_probe.py > $O/pinned_probe.log 2>&1 || exit 1
cat $O/pinned_probe.log
timeout -k 10 900 python -u scripts/edges_sweep.py --events 12500000 --variants default s512 s1024 s128 default --timeout 200 > $O/edges_12m.log 2>&1; rc=$?
cat $O/edges_12m.log; exit $rc
