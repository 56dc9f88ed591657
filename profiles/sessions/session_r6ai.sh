# cold ml_ops under glibc malloc settings (THP-backed malloc heap, fewer arenas): the ~1 GB of ordinary
# anonymous memory at exit costs kernel teardown time after os._exit (r6ag / r6ah)
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ai
mkdir -p $O
timeout -k 10 700 python -u scripts/cold_start.py --reps 4 --variants "default;GLIBC_TUNABLES=glibc.malloc.hugetlb=1;MALLOC_ARENA_MAX=4" --md $O/cold_malloc.md --json $O/cold_malloc.json > $O/cold_malloc.log 2>&1 || exit 1
grep median $O/cold_malloc.md
python - <<'PY'
import json
d = json.load(open("gpurun_out/r6ai/cold_malloc.json"))
for r in d["runs"]:
    m = r["marks"]
    print(r["variant"], r["wall_s"], "exit_call", m.get("exit_call"), "teardown", round(r["wall_s"] - m.get("exit_call", 0), 3), r.get("exit"))
PY
