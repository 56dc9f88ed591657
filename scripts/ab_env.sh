#!/bin/bash
# A/B of bench.py's ms per EM iteration under environment variants, interleaved to cancel drift:
#   bash scripts/ab_env.sh ROUNDS "ENV_A" "ENV_B" ... -- [bench args]
#   bash scripts/ab_env.sh 3 "ONI_GS_STAGE=4" "ONI_GS_STAGE=0" -- --steps 20 --warmup 5
set -u -o pipefail
rounds=$1; shift
variants=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do variants+=("$1"); shift; done
[ $# -gt 0 ] && shift
args=("$@")
for r in $(seq 1 "$rounds"); do
  for v in "${variants[@]}"; do
    out=$(env $v timeout -k 10 300 python -u bench.py --converge 0 --e2e 0 --e2e-cold 0 "${args[@]}" 2>/dev/null | grep '^{') || { echo "variant $v failed"; exit 1; }
    ms=$(echo "$out" | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "round $r  $v  ms_per_step=$ms"
  done
done
