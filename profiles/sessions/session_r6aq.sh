# DNS host cuts through the native ECDF in the forked prefetch child: GPU pipeline tests, DNS cold A/B vs HEAD
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export TAG=r6aq PYTEST_FILES=tests/test_gpu_pipeline.py
bash scripts/gpu.sh tests || exit $?
O=gpurun_out/r6aq
timeout -k 10 800 python -u scripts/cold_start.py --source dns --events 2000000 --reps 3 --variants "default;ROOT=abvar/base" --md $O/cold_dns_ab.md --json $O/cold_dns_ab.json > $O/cold_dns_ab.log 2>&1 || exit 1
grep median $O/cold_dns_ab.md
python - <<'PY'
import json, statistics as S
d = json.load(open("gpurun_out/r6aq/cold_dns_ab.json"))
by = {}
for r in d["runs"][1:]:
    m = r["marks"]; st = r["stages"]
    by.setdefault(r["variant"], []).append([r["wall_s"], m["torch_imported"], m["pipeline_end"]-m["pipeline_start"]] + [st[k] for k in ("load","dns_pre","lda","dns_post")])
for v, rows in by.items():
    print(v[:18].ljust(20), " ".join("%.3f" % S.median(c) for c in zip(*rows)), "(wall torch pipe load dns_pre lda dns_post)")
PY
