# 8 ranks sharing one GPU (12.5 M events, K = 100): per-rank cProfile of both host-resource variants
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out/r6s; mkdir -p $O
timeout -k 10 900 python -u scripts/pipeline_ranks.py --events 12500000 --days 4 --topics 100 --compat fixed \
  --tol 2.93e-8 --lag 0 --ranks 8 --threads 0 --timeout 400 \
  --variants "ONI_PROFILE=cprofile:$O/pa_{rank}.out;ONI_THREADS=16,ONI_PROFILE=cprofile:$O/pb_{rank}.out" \
  --json $O/ranks.json --md $O/ranks.md > $O/ranks.log 2>&1; rc=$?
for v in pa pb; do for r in 0 1; do python -c "import pstats; pstats.Stats('$O/${v}_$r.out').sort_stats('tottime').print_stats(20)" > $O/${v}_$r.txt 2>&1; done; done
nproc > $O/host.txt; cat /sys/fs/cgroup/cpu.max >> $O/host.txt 2>&1; cat /sys/fs/cgroup/cpuset.cpus.effective >> $O/host.txt 2>&1; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/host.txt
cat $O/ranks.md | head -30; head -30 $O/pa_1.txt; exit $rc
