#!/usr/bin/env python
"""Where LDAEngine construction spends its time (it is inside bench.py's to-convergence clock).

Builds the synthetic headline day, constructs the engine three times (the first loads code objects)
and prints the wall time of each plus the top functions of the last under cProfile.

  python scripts/setup_profile.py [--events 1000000] [--topics 20]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import torch
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    c, _ = synthetic_flow_corpus(events=a.events, seed=0, device="cuda")
    for rep in range(3):
        torch.cuda.synchronize()
        pr = cProfile.Profile() if rep == 2 else None
        t0 = time.perf_counter()
        if pr:
            pr.enable()
        eng = LDAEngine(c, a.topics, LDASettings(), backend="hip", seed=1, precision="fp64")
        torch.cuda.synchronize()
        if pr:
            pr.disable()
        print(f"construction {rep}: {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)
        del eng
    for key in ("cumulative", "tottime"):
        st = io.StringIO()
        pstats.Stats(pr, stream=st).sort_stats(key).print_stats(a.top)
        print(st.getvalue())


if __name__ == "__main__":
    main()
