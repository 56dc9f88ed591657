#!/usr/bin/env python
"""Where the to-convergence run's time goes beyond the steady-state iterations (headline corpus):
engine construction, init_random, the first iteration (graph capture), the rest of the EM loop."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    c, _ = synthetic_flow_corpus(events=1_000_000, seed=0, device="cuda")
    out = []
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng = LDAEngine(c, 20, LDASettings(), backend="hip", seed=1 + rep, precision="fp64")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        eng.init_random()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        r1 = eng.em_iterations_pipelined([1], True, c.num_docs)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        recs = eng.em_iterations_pipelined([8] * 13, True, c.num_docs, likelihood_old=r1[-1][0], iteration=1)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        n = 1 + len(recs)
        eng2 = LDAEngine(c, 20, LDASettings(), backend="hip", seed=1 + rep, precision="fp64")
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        res = eng2.run()
        torch.cuda.synchronize()
        t6 = time.perf_counter()
        out.append(dict(construct_ms=round((t1 - t0) * 1e3, 2), init_random_ms=round((t2 - t1) * 1e3, 2),
                        first_iter_ms=round((t3 - t2) * 1e3, 2), rest_ms=round((t4 - t3) * 1e3, 2), iters=n,
                        rest_per_iter_ms=round((t4 - t3) * 1e3 / max(n - 1, 1), 3),
                        run_ms=round((t6 - t5) * 1e3, 2), run_iters=res.em_iterations))
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
