# cold-start probes: anonymous mappings of a cold ml_ops process at exit; first launch of the framework's code
# object; process teardown by state (THP setting of the box)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ag
mkdir -p $O
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $O/thp.txt 2>&1 || true
cat $O/thp.txt
timeout -k 10 300 python -u scripts/micro/exit_smaps.py --out $O/exit_smaps.txt > $O/exit_smaps.log 2>&1 || exit 1
head -32 $O/exit_smaps.txt
timeout -k 10 200 python -u scripts/micro/first_op_cost.py --ops onihip_first,sort_i64,cumsum_i64,index_select,index_put --out $O/first_op_cost.json > $O/first_op_cost.log 2>&1 || exit 1
cat $O/first_op_cost.log
timeout -k 10 300 python -u scripts/micro/exit_teardown.py --reps 2 --out $O/exit_teardown.json > $O/exit_teardown.log 2>&1 || exit 1
tail -1 $O/exit_teardown.log
