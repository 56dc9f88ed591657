# sortgroup (no torch.unique / repeat_interleave / maximum / nonzero / bincount / float64 sort in the cold
# path) + native word names: all GPU tests, then the cold ml_ops A/B against HEAD's package (abvar/base)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6af
bash scripts/gpu.sh tests || exit $?
O=gpurun_out/r6af
timeout -k 10 600 python -u scripts/cold_start.py --reps 4 --variants "default;ROOT=abvar/base" --md $O/cold_ab.md --json $O/cold_ab.json > $O/cold_ab.log 2>&1 || exit 1
head -14 $O/cold_ab.md
grep median $O/cold_ab.md
timeout -k 10 300 python -u scripts/micro/exit_teardown.py --reps 3 --out $O/exit_teardown.json > $O/exit_teardown.log 2>&1 || exit 1
tail -1 $O/exit_teardown.log
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag || true
