#!/usr/bin/env python
"""Phase timing of the block E-step kernels (B4 / B8) and the split-document kernel on the 1-day
netflow corpus: thread 0 of block 0 (the bucket's longest document) accumulates clock64() cycles
per phase of the variational loop -- word pass, cross-lane/LDS reductions, barrier wait, topic
phase (wave 0); split: word pass, reductions, publish, gather wait, topic phase, loop barrier.

  python scripts/estep_phases.py [--topics K]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--events", type=int, default=1_000_000)
    a = ap.parse_args()
    from oni_ml_amd.models.lda import special
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.ops import hip as H
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    c, _ = synthetic_flow_corpus(events=a.events, seed=0, device="cuda")
    eng = LDAEngine(c, a.topics, LDASettings(), backend="hip", seed=0)
    eng.init_random()
    for _ in range(3):
        eng.em_iteration(True, c.num_docs)
    torch.cuda.synchronize()
    dc = eng.dc
    lc = special.lik_const(eng.alpha, eng.K)
    sp = eng.doc_buckets.split
    if sp is not None and not sp.wide:
        for bi, batch in enumerate(sp.batches):
            dbg = torch.zeros(8, dtype=torch.int64, device="cuda")
            H.lda_estep_split(dc.doc_ptr, dc.word_idx, dc.counts, eng.beta, eng.K, eng.alpha, lc, eng.var_max_iter,
                              eng.settings.var_converged, eng.gamma, eng.e, eng.r, eng.lik, eng.ass, eng.iters, batch,
                              sp.seg_words, dbg=dbg)
            torch.cuda.synchronize()
            d = dbg.cpu().tolist()
            it = max(d[6], 1)
            ph = ("word_pass", "reductions", "publish", "gather_wait", "topic_phase", "loop_barrier")
            print(json.dumps(dict(bucket=f"split[{bi}]", segments=d[7], blocks=int(batch["n_blocks"]), iterations=d[6],
                                  cycles_per_iteration={n: d[i] // it for i, n in enumerate(ph)},
                                  total_cycles=sum(d[:6]))), flush=True)
    names = {H.ESTEP_B4: "B4", H.ESTEP_B8: "B8"}
    for var, order in eng.doc_buckets.plan:
        if var not in names:
            continue
        dbg = torch.zeros(8, dtype=torch.int64, device="cuda")
        H.lda_estep(dc.doc_ptr, dc.word_idx, dc.counts, order, eng.beta, eng.K, eng.alpha, lc, eng.var_max_iter,
                    eng.settings.var_converged, eng.gamma, eng.e, eng.r, eng.lik, eng.ass, eng.iters, var, dbg=dbg)
        torch.cuda.synchronize()
        d = dbg.cpu().tolist()
        it = max(d[4], 1)
        print(json.dumps(dict(bucket=names[var], words=d[5], iterations=d[4],
                              cycles_per_iteration=dict(word_pass=d[0] // it, reductions=d[1] // it,
                                                        barrier=d[2] // it, topic_phase=d[3] // it),
                              total_cycles=sum(d[:4]))), flush=True)


if __name__ == "__main__":
    main()
