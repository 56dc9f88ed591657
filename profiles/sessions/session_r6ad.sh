# cold-start probes: process teardown after os._exit by device state; first-call cost of the pre stages' torch ops
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ad
mkdir -p $O
timeout -k 10 300 python -u scripts/micro/exit_teardown.py --reps 3 --out $O/exit_teardown.json > $O/exit_teardown.log 2>&1 || exit 1
tail -1 $O/exit_teardown.log
timeout -k 10 120 python -u scripts/micro/first_op_cost.py > $O/first_op_cost.log 2>&1 || exit 1
cat $O/first_op_cost.log
timeout -k 10 120 python -u scripts/micro/first_op_cost.py > $O/first_op_cost2.log 2>&1 || exit 1
tail -1 $O/first_op_cost2.log
