# cold ml_ops A/B: host cuts (hashed runs) after `import torch` (default) / the same cuts beside the import (abvar/base) /
# device cuts (abvar/nocuts)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ao
mkdir -p $O
timeout -k 10 800 python -u scripts/cold_start.py --reps 5 --variants "default;ROOT=abvar/base;ROOT=abvar/nocuts" --md $O/cold_ab.md --json $O/cold_ab.json > $O/cold_ab.log 2>&1 || exit 1
grep median $O/cold_ab.md
python - <<'PY'
import json, statistics as S
d = json.load(open("gpurun_out/r6ao/cold_ab.json"))
by = {}
for r in d["runs"][1:]:
    m = r["marks"]
    by.setdefault(r["variant"], []).append((r["wall_s"], m["torch_imported"], m["pipeline_end"] - m["pipeline_start"], r["stages"]["flow_pre"], r["wall_s"] - m.get("exit_call", 0)))
for v, rows in by.items():
    cols = list(zip(*rows))
    print(v, "median wall %.3f torch %.3f pipe %.3f flow_pre %.3f teardown %.3f" % tuple(S.median(c) for c in cols))
PY
