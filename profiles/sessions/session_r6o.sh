# verdict r5 item 3: the 8-rank config-5 pipeline on one GPU, each rank sized for the whole host
# (ONI_THREADS=16: no binding, 16 threads per rank, the round-5 default) against the per-rank budget
# (utils/hostres.py: CPU binding, threads = the rank's share of the cgroup quota)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6o; mkdir -p $O
timeout -k 10 120 rocprofv3 --list-avail > $O/pmc_avail.txt 2>&1 || true
timeout -k 10 1100 python -u scripts/pipeline_ranks.py --events 100000000 --days 30 --topics 100 --compat fixed \
  --tol 2.93e-8 --lag 0 --ranks 8 --threads 0 --variants 'ONI_THREADS=16;' --timeout 480 \
  --json $O/ranks_c5.json --md $O/ranks_c5.md > $O/ranks_c5.log 2>&1; rc=$?
tail -5 $O/ranks_c5.log; exit $rc
