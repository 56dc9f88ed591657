# K=100 shard: split-plan knobs (per-bucket timing + E-step graph) -- one bench_gs64 run per setting
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/knobs
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/bench_gs64.py --events 12500000 --topics 100 --warm-em 3 --reps 3 > gpurun_out/knobs/$name.json 2>/dev/null || { echo "$name failed"; return 1; }
  echo "$name $(tail -1 gpurun_out/knobs/$name.json)"
}
run default ONI_X=0 && run g32 ONI_GS_SPLIT_G=32 && run batches2 ONI_GS_SPLIT_BATCHES=2 && run words256 ONI_GS_SPLIT_WORDS=256
