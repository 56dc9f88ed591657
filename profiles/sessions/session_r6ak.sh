# host ECDF cuts in the input prefetch: all GPU tests, flow_pre steps cold, cold ml_ops A/B against HEAD~
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6ak
bash scripts/gpu.sh tests || exit $?
O=gpurun_out/r6ak
timeout -k 10 700 python -u scripts/cold_start.py --reps 4 --variants "default;ROOT=abvar/base" --md $O/cold_ab.md --json $O/cold_ab.json > $O/cold_ab.log 2>&1 || exit 1
grep median $O/cold_ab.md
python - <<'PY'
import json
d = json.load(open("gpurun_out/r6ak/cold_ab.json"))
for r in d["runs"]:
    m = r["marks"]
    print(f'{r["variant"][:16]:18s} wall {r["wall_s"]} torch {m["torch_imported"]} pipe {m["pipeline_end"]-m["pipeline_start"]:.3f} exit+{r["wall_s"]-m.get("exit_call",0):.3f}', r["stages"])
PY
