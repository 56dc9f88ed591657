#!/usr/bin/env python
"""The CPU baseline of BASELINE.json, measured on both schedules (verdict r4 item 4).

The C++ oni-lda-c-semantics engine (`oni_ml_amd/_lib/lda`, csrc/native/lda_ref.cpp; 20 document shards =
the reference's 20 MPI ranks, ml_ops.sh:80) trains bench.py's headline corpus (synthetic 1-day netflow,
1 M events, seed 0; K = 20, alpha0 = 2.5, lda-c default settings) twice:

  * lda-c's literal per-word schedule (the reference algorithm);
  * the GPU engine's block schedule (`--gs-updates 32`: gamma / digamma refreshed 32 times per sweep),
    so bench.py's vs_baseline can be read against the same arithmetic the GPU runs.

Per schedule: docs x EM iterations / s over bench.py's window (iterations 4-23: 3 warm-up + 20 timed) and
to convergence.  Writes a JSON record (default profiles/r5_cpu_baseline.json).

  ONI_THREADS=8 python scripts/cpu_baseline.py [--events N] [--out FILE]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--out", default="profiles/r5_cpu_baseline.json")
    ap.add_argument("--schedules", default="0,32", help="gs_updates values (0 = lda-c's per-word schedule)")
    ap.add_argument("--exe", default=None, help="another build of the `lda` binary (e.g. an older commit's)")
    a = ap.parse_args()
    import torch
    from oni_ml_amd.io import ldac
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    c, _ = synthetic_flow_corpus(events=a.events, seed=0, device=torch.device("cpu"))
    exe = a.exe or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oni_ml_amd", "_lib", "lda")
    threads = os.environ.get("ONI_THREADS", "8")
    rec = dict(exe=exe, corpus=dict(events=a.events, docs=c.num_docs, terms=c.num_terms, nnz=c.nnz),
               topics=a.topics, threads=int(threads), cpu=os.cpu_count(), runs=[])
    with tempfile.TemporaryDirectory() as tmp:
        ldac.write_model_dat(os.path.join(tmp, "model.dat"), c)
        with open(os.path.join(tmp, "settings.txt"), "w") as f:
            f.write(LDASettings().dumps())
        for u in (int(x) for x in a.schedules.split(",")):
            out = os.path.join(tmp, f"out{u}")
            cmd = [exe, "est", "2.5", str(a.topics), os.path.join(tmp, "settings.txt"), "20",
                   os.path.join(tmp, "model.dat"), "random", out] + (["--gs-updates", str(u)] if u else [])
            t0 = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, env=dict(os.environ, ONI_THREADS=threads))
            wall = time.perf_counter() - t0
            if r.returncode != 0:
                raise SystemExit(r.stderr)
            secs = [float(x) for x in re.findall(r"\*\*\*\* em iteration \d+ .* ([0-9.]+)s", r.stdout)]
            win = secs[3:23]
            run = dict(gs_updates=u, schedule="lda-c per-word" if u == 0 else f"block Gauss-Seidel, U = {u}",
                       em_iterations=len(secs), em_seconds=round(sum(secs), 3), wall_seconds=round(wall, 3),
                       window_iterations="4-23", window_s_per_iter=round(sum(win) / max(len(win), 1), 4),
                       window_docs_per_sec=round(c.num_docs * len(win) / max(sum(win), 1e-9)),
                       to_convergence_docs_per_sec=round(c.num_docs * len(secs) / max(sum(secs), 1e-9)),
                       command=" ".join([f"ONI_THREADS={threads} lda est 2.5 {a.topics} settings.txt 20 model.dat "
                                         "random out"] + cmd[9:]))
            rec["runs"].append(run)
            print(json.dumps(run), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
