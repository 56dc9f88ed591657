"""Host-side cost of enqueueing one EM iteration (graph replay vs eager launches) and the
device time per iteration for different read-back batch sizes.  Run on the GPU box."""
import json
import time

import torch

from oni_ml_amd.models.lda.em import LDAEngine
from oni_ml_amd.models.lda.settings import LDASettings
from oni_ml_amd.pipeline.flow import synthetic_flow_corpus


def main():
    c, _ = synthetic_flow_corpus(events=1_000_000, seed=0, device="cuda")
    out = {}
    for graph in (True, False):
        eng = LDAEngine(c, 20, LDASettings(), backend="hip", seed=0, use_graph=graph)
        eng.init_random()
        for _ in range(3):
            eng.em_iterations(5, True, c.num_docs, stop=False)
        torch.cuda.synchronize()
        key = "graph" if graph else "eager"
        # host enqueue time of 5 iterations (no read-back): replay / launch calls only
        t0 = time.perf_counter()
        if graph:
            (m, g), = eng._fgraphs.items()    # graphs of m = LDAEngine.graph_iters iterations (default 1)
            for _ in range(5 // m):
                g.replay()
        else:
            for _ in range(5):
                eng._launch_estep(newton_key=(True, c.num_docs))
        t_host = (time.perf_counter() - t0) / 5
        torch.cuda.synchronize()
        t_all = (time.perf_counter() - t0) / 5
        out[key] = dict(host_enqueue_ms=round(t_host * 1e3, 4), enqueue_plus_drain_ms=round(t_all * 1e3, 4))
        for b in (1, 5, 20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(max(1, 20 // b)):
                eng.em_iterations(b, True, c.num_docs, stop=False)
            torch.cuda.synchronize()
            out[key][f"ms_per_iter_batch{b}"] = round((time.perf_counter() - t0) / (max(1, 20 // b) * b) * 1e3, 4)
        del eng
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
