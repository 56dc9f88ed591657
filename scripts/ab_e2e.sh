#!/bin/bash
# A/B of bench.py's e2e ml_ops wall-clock (N = 1) under environment variants, interleaved:
#   bash scripts/ab_e2e.sh ROUNDS "ENV_A" "ENV_B" ...
set -u -o pipefail
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    out=$(env $v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --converge 0 2>/dev/null | grep '^{') || { echo "variant $v failed"; exit 1; }
    echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r  $v  e2e_wall_s=%s cold=%s stages=%s' % (d['e2e_wall_s'], d.get('e2e_cold_wall_s'), d['e2e_stage_s']))"
  done
done
