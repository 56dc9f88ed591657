# which stage of a cold ml_ops process maps the six ~173 MB anonymous regions seen at its exit (r6ag)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ah
mkdir -p $O
timeout -k 10 300 python -u scripts/micro/exit_smaps.py --out $O/exit_smaps.txt > $O/exit_smaps.log 2>&1 || exit 1
head -16 $O/exit_smaps.txt
cat $O/exit_smaps.txt.stages
timeout -k 10 300 python -u scripts/micro/cold_self_time.py --out $O/cold_self_time.md > $O/cold_self_time.log 2>&1 || exit 1
head -40 $O/cold_self_time.md
