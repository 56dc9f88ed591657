#!/usr/bin/env python
"""Where a cold `ml_ops` process spends its time (verdict r3 item 2: the cold ml_ops wall-clock).

Runs `python -m oni_ml_amd ml_ops 20160122 flow TOL` as fresh child processes on a synthetic day, as
bench.py's cold leg does (ml_ops.sh times each stage as a fresh process: ml_ops.sh:57,67,80,84,108):

  1. a first child (it fills the per-user bytecode cache, utils/pycache.py), then REPS rounds of the
     start-up variants (--variants, alternating): spawn -> exit wall, the start-up marks (interpreter, `import torch`, package,
     HIP context, pipeline start / end; cli.startup_marks) and the stage seconds;
  2. one run under `-X importtime`: the slowest imports (cumulative);
  3. one run under cProfile (ONI_PROFILE=cprofile:FILE): the host functions with the most cumulative time.

  python scripts/cold_start.py [--events 1000000] [--reps 3] [--md out.md] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import pstats
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


INPUT = []     # the source's input flags (main)


def _child(tmp, tag, tol, extra_env=None, pyflags=(), source="flow"):
    lpath = os.path.join(tmp, tag)
    extra_env = dict(extra_env or {})
    root = os.path.abspath(extra_env.pop("ROOT", ROOT))   # a variant's own copy of the package (A/B of host code)
    env = dict(os.environ, PYTHONPATH=root, **extra_env)
    for k in ("FLOW_PATH", "DNS_PATH", "LPATH", "TOL"):
        env.pop(k, None)
    args = ["20160122", source, repr(tol), "--lpath", lpath, "--conf", os.path.join(tmp, "none.conf"), "--quiet"] + INPUT
    launcher = os.path.join(root, "scripts", "ml_ops.sh")
    if pyflags or not os.path.exists(launcher):
        cmd = [sys.executable, *pyflags, "-m", "oni_ml_amd", "ml_ops"] + args
    else:   # the deployment launcher (its process environment included), as bench.py's cold leg
        cmd = ["bash", launcher] + args
    mark = os.path.join(lpath, ".exit_mark")
    t_spawn = time.time()
    env["ONI_T_SPAWN"] = repr(t_spawn)
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"{tag}: rc {r.returncode}\n{r.stderr[-3000:]}")
    with open(os.path.join(lpath, "run_summary.json")) as f:
        sm = json.load(f)
    try:   # the os._exit call (FAST_EXIT): what is left of the wall after it is process teardown
        with open(mark) as f:
            ex = f.read().split()
        sm.setdefault("startup_marks", {})["exit_call"] = round(float(ex[0]) - t_spawn, 4)
        sm["exit_status"] = dict(kv.split("=", 1) for kv in ex[1:])
    except (OSError, ValueError):
        pass
    return wall, sm, r.stderr


def _variants(spec):
    out = []
    for v in spec.split(";"):
        v = v.strip()
        # KEY=VALUE settings; ROOT=<dir>: run that directory's copy of the package
        env = {} if v in ("", "default") else dict(kv.split("=", 1) for kv in v.split())
        out.append((v or "default", env))
    return out


def _importtime(stderr, top):
    rows = []
    for line in stderr.splitlines():
        if not line.startswith("import time:") or "|" not in line:
            continue
        parts = line[len("import time:"):].split("|")
        try:
            rows.append((int(parts[1]), int(parts[0]), parts[2].rstrip()))
        except ValueError:
            continue
    rows.sort(reverse=True)
    # top-level packages only (the cumulative time of nested ones is inside their parent's)
    out = [(c, s, n) for c, s, n in rows if not n.startswith("    ")][:top]
    return [dict(module=n.strip(), cumulative_ms=round(c / 1e3, 1), self_ms=round(s / 1e3, 1)) for c, s, n in out]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tol", type=float, default=None, help="default 1e-5 (flow), 1e-4 (dns)")
    ap.add_argument("--source", default="flow", choices=["flow", "dns"])
    ap.add_argument("--md")
    ap.add_argument("--json")
    ap.add_argument("--variants", default="default;ONI_PYCACHE=0;ONI_FAST_EXIT=0;ONI_PREFETCH=0",
                    help="';'-separated env settings (space-separated KEY=VALUE within one), 'default' = none")
    ap.add_argument("--prof-out", help="keep the cProfile file here")
    a = ap.parse_args()
    from oni_ml_amd.synth.flow import generate_flow_day
    tmp = tempfile.mkdtemp(prefix="oni_cold_")
    try:
        if a.source == "flow":
            generate_flow_day(os.path.join(tmp, "in/"), events=a.events, seed=7)
            INPUT[:] = ["--flow-path", os.path.join(tmp, "in")]
        else:
            from oni_ml_amd.synth.dns import generate_dns_day
            g = generate_dns_day(os.path.join(tmp, "in"), events=a.events, seed=7, files=4,
                                 n_names=max(20_000, a.events // 10), n_clients=max(5_000, a.events // 40),
                                 with_edge_rows=False)
            INPUT[:] = ["--dns-path", g["dns_path"], "--top1m", g["top1m"]]
        a.tol = a.tol if a.tol is not None else (1e-5 if a.source == "flow" else 1e-4)
        runs = []
        # the variants alternate, so every one sees the same box state; the first child of all also fills
        # the per-user bytecode cache (utils/pycache.py) -- recorded as its own row, "first"
        variants = [("first", {})] + [v for _ in range(a.reps) for v in _variants(a.variants)]
        for i, (tag, env) in enumerate(variants):
            wall, sm, _ = _child(tmp, f"run{i}", a.tol, extra_env=env, source=a.source)
            runs.append(dict(variant=tag, wall_s=round(wall, 3), inprocess_s=round(sm["wall_seconds"], 3),
                             marks=sm.get("startup_marks"), exit=sm.get("exit_status"),
                             stages={k: round(v, 3) for k, v in sm["stage_seconds"].items()},
                             flagged=sm.get("scored")))
            print(json.dumps(runs[-1]), flush=True)
        _, _, err = _child(tmp, "importtime", a.tol, pyflags=("-X", "importtime"), source=a.source)
        imports = _importtime(err, 15)
        prof = os.path.join(tmp, "cold.prof")
        _child(tmp, "cprofile", a.tol, extra_env=dict(ONI_PROFILE=f"cprofile:{prof}"), source=a.source)
        if a.prof_out:
            shutil.copy(prof, a.prof_out)
        st = pstats.Stats(prof)
        st.sort_stats("cumulative")
        fn = []
        for (f, line, name), (cc, nc, tt, ct, callers) in sorted(st.stats.items(), key=lambda kv: -kv[1][3])[:40]:
            fn.append(dict(function=f"{os.path.relpath(f, ROOT) if f.startswith(ROOT) else os.path.basename(f)}:{line}({name})",
                           cumulative_s=round(ct, 4), self_s=round(tt, 4), calls=nc))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    rec = dict(events=a.events, runs=runs, imports=imports, cprofile=fn)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rec, f, indent=1)
    if a.md:
        L = [f"# Cold `ml_ops` process, 1-day {a.source} ({a.events} events)", "",
             "| run | variant | spawn -> exit s | in-process s | start-up marks (s after spawn) | stages s | flagged | at exit (kB) |",
             "|---|---|---|---|---|---|---|---|"]
        for i, r in enumerate(runs):
            L.append(f"| {i} | {r['variant']} | {r['wall_s']} | {r['inprocess_s']} | {r['marks']} | {r['stages']} | "
                     f"{r['flagged']} | {r.get('exit')} |")
        for v in dict.fromkeys(r["variant"] for r in runs):
            w = sorted(r["wall_s"] for r in runs if r["variant"] == v)
            L.append(f"\nmedian spawn -> exit, {v}: {w[len(w) // 2]} s ({len(w)} runs)")
        L += ["", "## Slowest imports (-X importtime, cumulative)", "", "| module | cumulative ms | self ms |",
              "|---|---|---|"]
        L += [f"| `{m['module']}` | {m['cumulative_ms']} | {m['self_ms']} |" for m in imports]
        L += ["", "## Host profile of the whole command (cProfile, cumulative)", "",
              "| function | cumulative s | self s | calls |", "|---|---|---|---|"]
        L += [f"| `{x['function']}` | {x['cumulative_s']} | {x['self_s']} | {x['calls']} |" for x in fn]
        with open(a.md, "w") as f:
            f.write("\n".join(L) + "\n")


if __name__ == "__main__":
    main()
