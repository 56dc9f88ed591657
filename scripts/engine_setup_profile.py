#!/usr/bin/env python
"""Where the LDA engine's construction goes on the headline corpus (bench.py's to-convergence clock
includes it): constructs LDAEngine 5 times (the first is the warm-up) and reports the median wall, then
once under cProfile (host functions by cumulative time; device work shows up as the synchronising calls).

  python scripts/engine_setup_profile.py [--topics 20] [--events 1000000] [--out gpurun_out/setup.txt]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    dev = torch.device("cuda")
    c, _ = synthetic_flow_corpus(events=a.events, seed=0, device=dev)
    walls = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng = LDAEngine(c, a.topics, LDASettings(), backend="hip", device=dev, seed=0)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        del eng
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    eng = LDAEngine(c, a.topics, LDASettings(), backend="hip", device=dev, seed=0)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    out = f"construction wall (ms): {[round(w * 1e3, 2) for w in walls]}\n" + s.getvalue()
    print(out)
    if a.out:
        with open(a.out, "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
