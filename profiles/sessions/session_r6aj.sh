# flow_pre step by step in a fresh process (cold vs warm); the cold ml_ops through the launcher (THP malloc)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6aj
mkdir -p $O
timeout -k 10 300 python -u scripts/micro/cold_flow_pre.py > $O/cold_flow_pre.md 2> $O/cold_flow_pre.err || { tail -20 $O/cold_flow_pre.err; exit 1; }
cat $O/cold_flow_pre.md
timeout -k 10 600 python -u scripts/cold_start.py --reps 3 --variants "default;GLIBC_TUNABLES=glibc.malloc.hugetlb=0" --md $O/cold.md --json $O/cold.json > $O/cold.log 2>&1 || exit 1
grep median $O/cold.md
