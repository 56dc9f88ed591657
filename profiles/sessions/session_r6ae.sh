# cold-start probes: first-call cost of each torch op in a fresh process; cold ml_ops with RSS / threads at exit
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ae
mkdir -p $O
timeout -k 10 300 python -u scripts/micro/first_op_cost.py --out $O/first_op_cost.json > $O/first_op_cost.log 2>&1 || exit 1
cat $O/first_op_cost.log
timeout -k 10 400 python -u scripts/cold_start.py --reps 2 --variants "default" --md $O/cold.md --json $O/cold.json > $O/cold.log 2>&1 || exit 1
head -8 $O/cold.md
