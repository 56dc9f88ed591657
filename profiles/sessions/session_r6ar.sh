# to-convergence run under EM batch sizes 8 / 4 / 2 / 1 (gated no-op iterations after convergence)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ar
mkdir -p $O
timeout -k 10 400 python -u scripts/micro/converge_batch_ab.py --reps 7 > $O/converge_batch_ab.log 2>&1 || { tail -20 $O/converge_batch_ab.log; exit 1; }
grep batch $O/converge_batch_ab.log
