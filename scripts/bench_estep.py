#!/usr/bin/env python
"""Per-bucket timing of the HIP E-step on the synthetic 1-day netflow corpus.

For each length bucket (and each split-document batch) it reports the number of
documents, their length range, variational iterations (mean / max) and the
kernel time measured with HIP events (median of repeats, one bucket at a time on
one stream), plus the suff-stats and M-step kernels and the whole EM step.

  python scripts/bench_estep.py [--events N] [--topics K] [--split-min W ...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--split-min", type=int, nargs="*", default=[1024, 4096, 1 << 30])
    ap.add_argument("--warm-em", type=int, default=3)
    ap.add_argument("--streams", type=int, nargs="+", default=[4], help="E-step stream counts to compare")
    a = ap.parse_args()
    from oni_ml_amd.models.lda import special
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.ops import hip as H
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    c, info = synthetic_flow_corpus(events=a.events, seed=0, device="cuda")
    lens = c.lengths()
    print(json.dumps(dict(docs=c.num_docs, nnz=c.nnz, V=c.num_terms, max_len=int(lens.max()),
                          len_pct={p: int(np.percentile(lens, p)) for p in (50, 90, 99, 99.9)})), flush=True)
    for smin in a.split_min:
        eng = LDAEngine(c, a.topics, LDASettings(), backend="hip", seed=0, split_min=smin, streams=a.streams[0])
        eng.init_random()
        for _ in range(a.warm_em):
            sc = eng.e_step()
            host = sc.cpu().tolist()
            eng.m_step(True, host[1], c.num_docs)
        torch.cuda.synchronize()
        dc = eng.dc
        lc = special.lik_const(eng.alpha, eng.K)
        it = eng.iters.cpu().numpy()
        rows = []
        sp = eng.doc_buckets.split
        if sp is not None:
            for bi, batch in enumerate(sp.batches):
                docs = batch["seg_doc"].cpu().numpy()
                ud = np.unique(docs)
                ms = timed(lambda: H.lda_estep_split(dc.doc_ptr, dc.word_idx, dc.counts, eng.beta, eng.K, eng.alpha, lc,
                                                     eng.var_max_iter, eng.settings.var_converged, eng.gamma, eng.e,
                                                     eng.r, eng.lik, eng.ass, eng.iters, batch, sp.seg_words,
                                                     wide=sp.wide))
                rows.append(dict(bucket=f"split[{bi}]", docs=int(ud.size), blocks=int(batch["n_blocks"]),
                                 len_min=int(lens[ud].min()), len_max=int(lens[ud].max()),
                                 it_mean=round(float(it[ud].mean()), 2), it_max=int(it[ud].max()), ms=round(ms, 4)))
        for var, order in eng.doc_buckets.plan:
            o = order.cpu().numpy()
            ms = timed(lambda: H.lda_estep(dc.doc_ptr, dc.word_idx, dc.counts, order, eng.beta, eng.K, eng.alpha, lc,
                                           eng.var_max_iter, eng.settings.var_converged, eng.gamma, eng.e, eng.r,
                                           eng.lik, eng.ass, eng.iters, var))
            rows.append(dict(bucket=["G16", "G32", "G64", "G64C", "B4", "B8", "T1", "W16", "W32", "W64", "WB4", "WB8"][var], docs=int(o.size),
                             len_min=int(lens[o].min()), len_max=int(lens[o].max()),
                             it_mean=round(float(it[o].mean()), 2), it_max=int(it[o].max()), ms=round(ms, 4)))

        def suff():
            H.lda_suffstats_fused(dc.word_ptr, dc.csc_ent, dc.csc_doc, eng.suff_plan, eng.e, eng.r, eng.beta, eng.cw,
                                  eng._suff_part, scalars=(eng.lik, eng.ass, 0, eng.lik.numel()))
            H.colsum_partials(eng._suff_part, eng.suff_plan.n_blocks, eng._red_local)
        rows.append(dict(bucket="suffstats", ms=round(timed(suff), 4)))
        rows.append(dict(bucket="mstep", ms=round(timed(lambda: eng.m_step(False, 0.0, c.num_docs)), 4)))

        def step():
            eng.em_iteration(True, c.num_docs)
        rows.append(dict(bucket="EM step (hipGraph)", ms=round(timed(step, 10), 4), var_max_iter=eng.var_max_iter,
                         streams=a.streams[0]))
        rows.append(dict(bucket="EM step (hipGraph, 5 per read-back)", streams=a.streams[0],
                         ms=round(timed(lambda: eng.em_iterations(5, True, c.num_docs, stop=False), 5) / 5, 4)))
        for ns in a.streams[1:]:
            e2 = LDAEngine(c, a.topics, LDASettings(), backend="hip", seed=0, split_min=smin, streams=ns)
            e2.init_random()
            for _ in range(a.warm_em):
                e2.em_iteration(True, c.num_docs)
            rows.append(dict(bucket="EM step (hipGraph)", streams=ns,
                             ms=round(timed(lambda: e2.em_iteration(True, c.num_docs), 10), 4)))
            del e2
        eng.use_graph = False
        rows.append(dict(bucket="EM step (eager launches)", ms=round(timed(step, 10), 4)))
        eng.use_graph = True
        print(json.dumps(dict(split_min=smin, rows=rows)), flush=True)


if __name__ == "__main__":
    main()
