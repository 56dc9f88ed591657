#!/usr/bin/env python
"""Per-bucket timing of the fp64 block Gauss-Seidel E-step (csrc/hip/lda_gs64.hip).

Trains a few EM iterations on the synthetic 1-day netflow corpus (bench.py's headline corpus),
then launches each length bucket alone (HIP events, median of repeats) and reports documents,
lengths, sweeps and kernel time; plus suff-stats and the M-step.  ``--only VARIANT`` loops one
bucket (for rocprofv3 --pmc runs of a single kernel).

  python scripts/bench_gs64.py [--events N] [--topics K] [--gs-updates U] [--only split|tiny|team1|team4|team8]
"""
import argparse
import json
import os
import sys

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
    ap.add_argument("--gs-updates", type=int, default=0)
    ap.add_argument("--warm-em", type=int, default=4)
    ap.add_argument("--only", default=None)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--phases", action="store_true", help="phase timer of the longest document of each team bucket")
    ap.add_argument("--first", type=int, default=0,
                    help="team buckets: only their FIRST longest documents (e.g. 1: the longest document alone)")
    ap.add_argument("--prefixes", default="", help="also time the team8 bucket on its N longest documents, e.g. 1,2,8")
    ap.add_argument("--xsplit", type=int, default=0, help="the N longest documents on the XCD-split kernel (gs_xsplit)")
    ap.add_argument("--xsplit-g", type=int, default=0, help="gs_xsplit members per document (0: the LDS minimum)")
    ap.add_argument("--long", default="", help="a synthetic corpus of only these document lengths (e.g. 443426: "
                                               "config 5's longest document alone), distinct random words")
    ap.add_argument("--vocab", type=int, default=4_536_586, help="--long: vocabulary (config 5's month)")
    ap.add_argument("--sweeps", type=int, default=0, help="timed launches run exactly this many sweeps (no "
                                                           "convergence test), e.g. 20: a long document's real count")
    a = ap.parse_args()
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.ops import hip as H
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    if a.long:
        from oni_ml_amd.corpus.csr import Corpus
        rng = np.random.default_rng(0)
        lens = np.asarray([int(x) for x in a.long.split(",")], np.int64)
        ptr = np.concatenate([[0], np.cumsum(lens)])
        words = np.concatenate([np.sort(rng.choice(a.vocab, n, replace=False)) for n in lens]).astype(np.int32)
        c = Corpus(ptr, words, rng.integers(1, 4, words.size).astype(np.int64), a.vocab)
    else:
        c, _ = synthetic_flow_corpus(events=a.events, seed=0, device="cuda")
    st = LDASettings()
    st.gs_updates = a.gs_updates
    xs = dict(docs=a.xsplit, members=a.xsplit_g) if a.xsplit else None
    eng = LDAEngine(c, a.topics, st, backend="hip", seed=0, precision="fp64", xsplit=xs)
    eng.init_random()
    eng.em_iterations(a.warm_em, True, c.num_docs, stop=False)
    torch.cuda.synchronize()
    if a.sweeps:
        # params {alpha, lgamma const, VAR_MAX_ITER, VAR_CONVERGED, ...}: fixed sweeps for the timed launches
        eng._params[2] = float(a.sweeps)
        eng._params[3] = -1e30
    dc = eng.dc
    lens = c.lengths()
    its = eng.iters.cpu().numpy()
    names = {H.GS_TINY: "tiny", H.GS_TEAM1: "team1", H.GS_TEAM4: "team4", H.GS_TEAM8: "team8", H.GS_SMALL: "small",

             H.GS_CHAIN: "chain"}
    out = dict(docs=c.num_docs, nnz=c.nnz, U=eng._U, buckets=[])

    def launch(var, order, dbg=None):
        st = eng._stages.get(id(order))   # team8's staged rows (ops/hip.py GSStage): refill + launch
        if st is not None:
            H.gs_stage(eng.beta, dc.word_idx, st)
        H.gs_estep(dc.doc_ptr, dc.word_idx, dc.counts, order, eng.beta, eng.K, eng._U, eng._params, eng.gamma,
                   eng.cphi, eng.lik, eng.ass, eng.iters, var, dbg=dbg, stage=st)

    spl = eng.gs_plan.split
    if spl is not None and (not a.only or a.only == "split"):
        def split_fn(b):
            return H.gs_xsplit if b.get("x") else H.gs_split

        def launch_split():
            for b in spl.batches:
                split_fn(b)(dc.doc_ptr, dc.word_idx, dc.counts, eng.beta, eng.K, eng._U, eng._params, eng.gamma,
                            eng.cphi, eng.lik, eng.ass, eng.iters, b)
        o = np.asarray(sorted(spl.segments), dtype=np.int64)
        L, it = lens[o], its[o]
        out["buckets"].append(dict(kernel="split", docs=int(o.size), len_min=int(L.min()), len_max=int(L.max()),
                                   entries=int(L.sum()), sweeps_mean=round(float(it.mean()), 2),
                                   sweeps_max=int(it.max()), ms=round(timed(launch_split, a.reps), 4),
                                   word_sweeps=int((L * it).sum()), batches=len(spl.batches),
                                   workgroups=int(sum(spl.segments.values())),
                                   max_segments=int(max(spl.segments.values()))))
        if a.phases:
            dbg = torch.zeros(8, dtype=torch.int64, device="cuda")
            b0 = spl.batches[0]
            split_fn(b0)(dc.doc_ptr, dc.word_idx, dc.counts, eng.beta, eng.K, eng._U, eng._params, eng.gamma,
                         eng.cphi, eng.lik, eng.ass, eng.iters, b0, dbg=dbg)
            v = dbg.cpu().tolist()
            if b0.get("x"):   # gs_xsplit: word + reduce, publish -> gathered, refresh, chunks
                ch = max(v[3], 1)
                d0 = int(spl.batches[0]["seg_doc"][(b0["seg_doc"] >= 0).nonzero()[0, 0]].item())
                out["buckets"][-1]["phase_cycles_per_chunk"] = dict(
                    word_reduce=round(v[0] / ch), exchange=round(v[1] / ch), refresh=round(v[2] / ch), chunks=v[3],
                    doc_len=int(lens[d0]), members=int(spl.segments[d0]),
                    placed=b0["placed"].cpu().tolist())
            else:
                ch = max(v[7], 1)
                d0 = int(b0["seg_doc"][0].item())
            if not b0.get("x"):
                out["buckets"][-1]["phase_cycles_per_chunk"] = dict(
                # gs_splitw tick indices: word waves 0-2, topic wave 3-6 (lda_gs64.hip)
                word=round(v[0] / ch), word_prefetch_issue=round(v[1] / ch), word_barrier_b=round(v[2] / ch),
                topic_wait_arrivals=round(v[3] / ch), exchange=round(v[4] / ch), refresh=round(v[5] / ch),
                sweep_end_total=v[6], chunks=v[7], doc_len=int(lens[d0]),
                segments=int(b0["seg_count"][0].item()))
        print(json.dumps(out["buckets"][-1]), flush=True)
    for var, order in eng.gs_plan.plan:
        if a.only and names[var] != a.only:
            continue
        o = order.cpu().numpy()
        o = o[o >= 0]   # XCD placement gaps
        if a.first and var in (H.GS_TEAM1, H.GS_TEAM4, H.GS_TEAM8):
            o = o[:a.first]
            keep = eng._stages.pop(id(order), None)
            order = torch.from_numpy(o.astype(np.int32)).to(order.device)
            if keep is not None:
                eng._stages[id(order)] = H.GSStage(order, c.doc_ptr, eng.KS, order.device)
        L = lens[o]
        ms = timed(lambda: launch(var, order), a.reps)
        it = its[o]
        out["buckets"].append(dict(kernel=names[var], docs=int(o.size), len_min=int(L.min()), len_max=int(L.max()),
                                   entries=int(L.sum()), sweeps_mean=round(float(it.mean()), 2),
                                   sweeps_max=int(it.max()), ms=round(ms, 4),
                                   word_sweeps=int((L * it).sum())))
        if a.phases and var not in (H.GS_TINY, H.GS_SMALL, H.GS_CHAIN):
            dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
            launch(var, order, dbg)
            v = dbg.cpu().tolist()
            ch = max(v[7], 1)
            out["buckets"][-1]["phase_cycles_per_chunk"] = dict(
                word=round(v[0] / ch), word_dot=round(v[6] / ch), reduce=round(v[1] / ch), barrier1=round(v[2] / ch), topic=round(v[3] / ch),
                barrier2=round(v[4] / ch), sweep_tail_total=v[5], chunks=v[7], doc_len=int(L.max()))
            if any(v[8:12]):   # gs_wsteam's topic wave
                out["buckets"][-1]["topic_wave_cycles_per_chunk"] = dict(
                    wait_arrivals=round(v[8] / ch), sum_refresh=round(v[9] / ch), barrier_b=round(v[10] / ch),
                    after_barrier=round(v[11] / ch), seen_wave0=round(v[12] / ch), seen_wave3=round(v[13] / ch),
                    seen_wave4=round(v[14] / ch), seen_last=round(v[15] / ch))
        st = eng._stages.get(id(order))
        if st is not None:
            out["buckets"][-1]["stage_ms"] = round(timed(lambda: H.gs_stage(eng.beta, dc.word_idx, st), a.reps), 4)
            out["buckets"][-1]["stage_mb"] = round(st.nbytes / 2**20, 1)
        print(json.dumps(out["buckets"][-1]), flush=True)
        if a.prefixes and var == H.GS_TEAM8:
            # the longest documents alone: separates the per-CU gather rate from L2 sharing between documents
            for npre in [int(x) for x in a.prefixes.split(",")]:
                sub = torch.from_numpy(o[:npre].copy()).to(order.device)
                print(json.dumps(dict(kernel="team8", prefix_docs=npre, len_max=int(L.max()),
                                      ms=round(timed(lambda: launch(var, sub), a.reps), 4))), flush=True)
    if not a.only:
        sp = eng.suff_plan
        out["suff_ms"] = round(timed(lambda: H.gs_suff64(dc.word_ptr, dc.csc_ent, sp, eng.cphi, eng.cw,
                                                         eng._suff_part, scalars=(eng.lik, eng.ass, 0, eng.D))), 4)
        out["estep_graph_ms"] = round(timed(lambda: eng._launch_estep()), 4)
        print(json.dumps({k: v for k, v in out.items() if k != "buckets"}), flush=True)


if __name__ == "__main__":
    main()
