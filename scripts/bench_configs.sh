#!/bin/bash
# BASELINE.json configs on one MI355X (per-GPU shard of the 8-GPU configs):
#   headline  flow 1-day, K=20
#   config 3  flow 1-day, K=50          (8 GPUs: one day per GPU, weak scaling)
#   config 4  DNS 1-day (2M queries), K=20
#   config 5  flow 30-day / 8 = 12.5M events per GPU, K=100
set -o pipefail
D=${OUTDIR:-gpurun_out}/cfg
mkdir -p $D
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 "$@" > $D/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -20 $D/$name.log; return 1; }
  grep '^{' $D/$name.log | tail -1 > $D/$name.json
  python - "$D/$name.json" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["config"]
print(f"{sys.argv[2]:10s} K={c['model'][-3:]} docs={c.get('docs', c.get('docs_per_gpu'))} V={c['vocab']} "
      f"nnz={c.get('nnz', c.get('nnz_per_gpu'))} "
      f"ms/iter={d['ms_per_step']} docs/s={d['value']:.3e} var_iter_mean={d.get('var_iter_mean')} "
      f"converge={d.get('converge_seconds')}s/{d.get('converge_em_iters')}it corpus_build={d.get('corpus_build_s')}s")
PY
}
run headline "$@" && \
run flow_k50 --topics 50 --e2e 0 --e2e-cold 0 "$@" && \
run dns_k20 --corpus dns --e2e 0 --e2e-cold 0 "$@" && \
run flow30d_k100 --topics 100 --events 12500000 --e2e 0 --e2e-cold 0 "$@"
