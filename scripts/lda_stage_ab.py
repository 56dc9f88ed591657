#!/usr/bin/env python
"""Why the ml_ops `lda` stage costs more than its EM (verdict r5 item 4): the warm flow pipeline on the
synthetic headline day, in this process, under variants that remove one suspect at a time:

  default      as shipped
  sync_pre     lda_pre's text files written before the lda stage (no writer thread beside the EM)
  lag0         no LAG model files inside the EM loop (only 000 and final)
  threads4     the background writers on 4 threads
  nowc         no doc_wc.dat (the lda_pre writer's one job that copies device tensors to the host)
  switch       the interpreter's GIL switch interval at 0.2 ms instead of 5 ms

Each variant runs --reps times after one untimed warm-up run; prints the median stage seconds and the
lda stage's own breakdown (estimate(): setup, EM loop, final pass).

  python scripts/lda_stage_ab.py [--events 1000000] [--variants default,sync_pre,lag0] [--reps 3]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--variants", default="default,sync_pre,lag0,threads4")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch
    from oni_ml_amd import config as CFG
    from oni_ml_amd.pipeline import common as C
    from oni_ml_amd.pipeline import run
    from oni_ml_amd.synth.flow import generate_flow_day
    tmp = tempfile.mkdtemp(prefix="oni_lda_ab_")
    generate_flow_day(os.path.join(tmp, "in/"), events=a.events, seed=7)
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    real_bg = C.background
    out = {}
    try:
        for v in ["warmup"] + a.variants.split(","):
            recs = []
            for rep in range(1 if v == "warmup" else a.reps):
                lp = os.path.join(tmp, f"ml_{v}_{rep}")
                os.makedirs(lp)
                cfg = CFG.resolve("20160122", "flow", tol=1e-5, conf_path=None, environ={}, lpath=lp,
                                  flow_path=os.path.join(tmp, "in"), verbose=False,
                                  threads=4 if v == "threads4" else None)
                if v == "lag0":
                    cfg.settings.lag = 0
                if v == "nowc":
                    cfg.write_doc_wc = False
                sys.setswitchinterval(2e-4 if v == "switch" else 5e-3)
                C.background = (lambda fn, name="": (fn(), (lambda: None))[1]) if v == "sync_pre" else real_bg
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                s = run(cfg, device=dev, log=lambda *x, **k: None)
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                wall = time.perf_counter() - t0
                tm = dict(s.get("lda", {}).get("timing", {}))
                tm.update({"host_" + k: x for k, x in tm.pop("em_host", {}).items()})
                recs.append(dict(wall=wall, stages=s.get("stage_seconds", {}), lda=tm))
                shutil.rmtree(lp, ignore_errors=True)
            C.background = real_bg
            if v == "warmup":
                continue
            med = lambda xs: round(float(np.median(xs)), 4)   # noqa: E731
            r = dict(wall=med([x["wall"] for x in recs]),
                     stages={k: med([x["stages"].get(k, 0.0) for x in recs]) for k in recs[0]["stages"]},
                     lda={k: med([x["lda"].get(k, 0.0) for x in recs]) for k in recs[0]["lda"]})
            out[v] = r
            print(json.dumps(dict(variant=v, **r)), flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
