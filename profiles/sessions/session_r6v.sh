# strong-scaling emulation of the 1-day configs on round-6 kernels (headline K = 20, config 3 K = 50, config 4 DNS);
# where a cold ml_ops child spends its time (cProfile kept)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6v STRONG_ARGS="--configs headline,k50,dns" COLD_ARGS="--reps 2 --variants default --prof-out gpurun_out/r6v/cold_prof.out"
bash scripts/gpu.sh cold strong
