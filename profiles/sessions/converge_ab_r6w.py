#!/usr/bin/env python
"""bench.py's to-convergence run (fresh engine + random init until lda-c's EM loop test stops it, engine
construction inside the clock) repeated under engine variants, interleaved so box drift hits both alike:

  python scripts/converge_ab.py --reps 7 [--variants default,noprelaunch]

  default       as shipped
  noprelaunch   LDAEngine.capture_prelaunch = False (the first graph captured right after one launch)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--variants", default="default,noprelaunch")
    ap.add_argument("--events", type=int, default=1_000_000)
    a = ap.parse_args()
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    c, _ = synthetic_flow_corpus(events=a.events, seed=0, device="cuda")
    vs = a.variants.split(",")
    res = {v: [] for v in vs}
    for rep in range(a.reps + 1):
        for v in vs:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng = LDAEngine(c, 20, LDASettings(), alpha_init=2.5, backend="hip", seed=1)
            if v == "noprelaunch":
                eng.capture_prelaunch = False
            torch.cuda.synchronize()
            ts = time.perf_counter() - t0
            r = eng.run()
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            if rep > 0:       # the first round loads code objects
                res[v].append(dict(s=t, setup=ts, iters=r.em_iterations, lik=r.likelihoods[-1][0]))
            del eng
    for v in vs:
        s = [x["s"] for x in res[v]]
        print(json.dumps(dict(variant=v, median_ms=round(1e3 * float(np.median(s)), 3), min_ms=round(1e3 * min(s), 3),
                              setup_ms=round(1e3 * float(np.median([x["setup"] for x in res[v]])), 3),
                              iters=res[v][0]["iters"], lik=res[v][0]["lik"],
                              all_ms=[round(1e3 * x, 2) for x in s])), flush=True)


if __name__ == "__main__":
    main()
