#!/usr/bin/env python
"""Precision and schedule parity of the GPU engines against lda-c on the headline bench corpus.

The reference core (oni-lda-c) computes in double with a per-word
Gauss-Seidel schedule.  This script trains the SAME corpus (bench.py's 1-day synthetic netflow,
seed 0) from the SAME random init with several engines and compares what the pipeline consumes:

  hip    fp64 block Gauss-Seidel (HIP kernels, csrc/hip/lda_gs64.hip; the bench path): gamma
         refreshed every ceil(n/32) words, lda-c's per-word schedule for documents <= 32 words
  torch  fp64 Jacobi E-step (PyTorch on the host CPU, ops/reference.py)
  cpu    fp64 Gauss-Seidel E-step, a literal transcription of lda-c's lda_inference
         (csrc/native/lda_ref.cpp; the engine BASELINE.json's docs/s was measured with)
  cpuU   the C++ engine with the GPU engine's block schedule (U = 32): the GPU engine's oracle

Compared: per-EM-iteration likelihood, EM iterations to convergence, final alpha, the
exported doc topics theta = gamma / sum(gamma) and word topics phi = softmax(log beta) rows
(lda_post.py semantics), and the scorer's ranking of (doc, word) entries by
theta_d . phi_w (flow_post_lda.scala:227-239: the lowest scores are the flagged events).

`cpu#20` is lda-c with its statistics reduced as 20 MPI ranks (the reference's process_count):
the reference's own floating-point spread from nothing but summation order.
A fourth run, `cpu@1`, is lda-c's own run-to-run spread: the same fp64 engine from another
random init (oni-lda-c seeds its MT19937 from the clock, so no two reference runs agree).

  python scripts/precision_parity.py [--events 1000000] [--topics 20] [--engines hip,torch,cpu,cpu@1]
  python scripts/precision_parity.py --corpus dns --events 2000000 --engines cpu,cpuU,cpu@1      (config 4)
  python scripts/precision_parity.py --events 12500000 --topics 100 --sub-nnz 1500000 --engines cpu,cpuU,cpu@1

``cpuU`` is the GPU engine's arithmetic and schedule (tests/test_gs64.py pins the HIP kernels to it at
1e-10), so a CPU-only run (cpu, cpuU, cpu@1) measures the GPU engine's parity with lda-c.
``--sub-nnz``: keep the longest documents (they carry the block schedule's largest chunks) plus a
seeded random sample of the others up to about that many corpus entries.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _train(corpus, K, name, dev, seed, var_max_iter=None):
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    st = LDASettings()
    if var_max_iter is not None:
        st.var_max_iter = var_max_iter
    name, _, shards = name.partition("#")       # "cpu#20": lda-c reduced as 20 MPI ranks
    backend = {"hip": "hip", "torch": "torch", "cpu": "cpu", "cpuU": "cpu"}[name]
    if name == "cpuU":
        st.gs_updates = GS_U
    eng = LDAEngine(corpus, K, st, backend=backend, device=dev, seed=seed)
    if shards:
        eng.cpu_shards = int(shards)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = eng.run(start="random", on_iteration=lambda e, i, L, c: print(f"  {name} it {i} L={L:.6f}", flush=True))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    sec = time.perf_counter() - t0
    res.gamma = np.asarray(eng.gather_gamma(), dtype=np.float64)
    res.log_beta = np.asarray(eng.log_beta(), dtype=np.float64)
    return res, sec


GS_U = 32


def _subsample(c, nnz, keep, seed):
    """The `keep` longest documents plus random others (corpus order kept) up to ~nnz entries; the
    vocabulary is re-indexed to the words that remain."""
    from oni_ml_amd.corpus.csr import Corpus
    lens = c.lengths()
    order = np.argsort(-lens, kind="stable")
    chosen = set(order[:keep].tolist())
    budget = nnz - int(lens[order[:keep]].sum())
    rng = np.random.default_rng(seed + 17)
    for d in rng.permutation(c.num_docs):
        if budget <= 0:
            break
        if d not in chosen:
            chosen.add(int(d))
            budget -= int(lens[d])
    docs = np.array(sorted(chosen), np.int64)
    ptr = np.concatenate([[0], np.cumsum(lens[docs])])
    idx = np.concatenate([np.arange(c.doc_ptr[d], c.doc_ptr[d + 1]) for d in docs])
    w = c.word_idx[idx]
    uw, inv = np.unique(w, return_inverse=True)
    return Corpus(ptr, inv.astype(np.int32), c.counts[idx], int(uw.size))


def _theta(gamma):
    s = gamma.sum(1, keepdims=True)
    return np.where(s > 0, gamma / np.where(s > 0, s, 1.0), 0.0)


def _phi(log_beta):
    x = log_beta - log_beta.max(1, keepdims=True)
    p = np.exp(x)
    return (p / p.sum(1, keepdims=True)).T          # [V, K]


def _entry_scores(corpus, theta, phi):
    doc = np.repeat(np.arange(corpus.num_docs), np.diff(corpus.doc_ptr))
    return np.einsum("ek,ek->e", theta[doc], phi[corpus.word_idx])


def _topk_overlap(a, b, k):
    ia = set(np.argsort(a, kind="stable")[:k].tolist())
    ib = set(np.argsort(b, kind="stable")[:k].tolist())
    return len(ia & ib) / k


def _tie_closed_overlap(a, b, k):
    """Overlap of the lowest-k sets with every entry TIED (exactly equal score, same run) with the k-th
    one included on both sides: |A* & B*| / min(|A*|, |B*|).  Entries of identical documents and words
    score identically, so a cut through a tie group picks an arbitrary (entry-id) part of it; when two
    runs order two near-equal groups differently, the plain overlap drops by a whole group."""
    ta, tb = np.sort(a, kind="stable")[k - 1], np.sort(b, kind="stable")[k - 1]
    ia, ib = np.flatnonzero(a <= ta), np.flatnonzero(b <= tb)
    return float(np.intersect1d(ia, ib).size / max(1, min(ia.size, ib.size))), int(ia.size), int(ib.size)


def _spearman(a, b):
    ra = np.empty(len(a)); ra[np.argsort(a, kind="stable")] = np.arange(len(a))
    rb = np.empty(len(b)); rb[np.argsort(b, kind="stable")] = np.arange(len(b))
    return float(np.corrcoef(ra, rb)[0, 1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--engines", default="hip,cpu,cpuU,cpu@1")
    ap.add_argument("--var-max-iter", type=int, default=None, help="override settings.txt var max iter (20)")
    ap.add_argument("--corpus", default="flow", choices=["flow", "dns"])
    ap.add_argument("--sub-nnz", type=int, default=0, help="sub-sample to ~this many entries, longest documents kept")
    ap.add_argument("--keep-longest", type=int, default=20)
    ap.add_argument("--gs-updates", type=int, default=32, help="U of the cpuU engine (the GPU schedule)")
    ap.add_argument("--json", default=None)
    ap.add_argument("--md", default=None)
    ap.add_argument("--save-scores", default=None, help="npz of every engine's entry scores (re-derive metrics later)")
    args = ap.parse_args()

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if args.corpus == "dns":
        from oni_ml_amd.pipeline.dns import synthetic_dns_corpus
        corpus, _ = synthetic_dns_corpus(events=args.events, seed=args.seed, device=dev)
    else:
        from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
        corpus, _ = synthetic_flow_corpus(events=args.events, seed=args.seed, device=dev)
    if args.sub_nnz and corpus.nnz > args.sub_nnz:
        corpus = _subsample(corpus, args.sub_nnz, args.keep_longest, args.seed)
    global GS_U
    GS_U = args.gs_updates
    print(f"corpus: {corpus.num_docs} docs, {corpus.num_terms} words, {len(corpus.word_idx)} entries", flush=True)

    runs = {}
    for name in args.engines.split(","):
        eng_name, _, seed = name.partition("@")       # "cpu@1": the cpu engine from another random init
        # the fp64 PyTorch Jacobi engine runs on the host: its per-bucket launches make it slower on the GPU
        d = dev if eng_name.startswith("hip") else torch.device("cpu")
        res, sec = _train(corpus, args.topics, eng_name, d, int(seed) if seed else args.seed, args.var_max_iter)
        runs[name] = dict(res=res, sec=sec)
        print(f"{name}: {res.em_iterations} EM iterations, {sec:.2f} s, L={res.likelihoods[-1][0]:.6f}, "
              f"alpha={res.alpha:.8f}", flush=True)

    names = list(runs)
    ref_name = "cpu" if "cpu" in runs else names[-1]
    derived = {}
    for name, r in runs.items():
        th, ph = _theta(r["res"].gamma), _phi(r["res"].log_beta)
        derived[name] = dict(theta=th, phi=ph, score=_entry_scores(corpus, th, ph),
                             L=np.array([x[0] for x in r["res"].likelihoods]))
    k_top = max(1, len(corpus.word_idx) // 1000)
    if args.save_scores:
        np.savez(args.save_scores, **{n.replace("@", "_at_").replace("#", "_x"): d["score"] for n, d in derived.items()})
    out = dict(corpus=dict(docs=corpus.num_docs, words=corpus.num_terms, entries=int(len(corpus.word_idx)),
                           events=args.events, seed=args.seed), topics=args.topics, engines={}, pairs={})
    for name, r in runs.items():
        res = r["res"]
        out["engines"][name] = dict(seconds=round(r["sec"], 3), em_iterations=res.em_iterations,
                                    final_likelihood=float(derived[name]["L"][-1]), alpha=float(res.alpha),
                                    likelihood_trajectory=[float(x) for x in derived[name]["L"]])
    for i, a in enumerate(names):
        for b in names[i + 1:]:
            A, B = derived[a], derived[b]
            n = min(len(A["L"]), len(B["L"]))
            out["pairs"][f"{a} vs {b}"] = dict(
                likelihood_rel_diff_max=float(np.max(np.abs(A["L"][:n] - B["L"][:n]) / np.abs(B["L"][:n]))),
                final_likelihood_rel_diff=float(abs(A["L"][-1] - B["L"][-1]) / abs(B["L"][-1])),
                alpha_rel_diff=float(abs(runs[a]["res"].alpha - runs[b]["res"].alpha) / runs[b]["res"].alpha),
                theta_max_abs_diff=float(np.abs(A["theta"] - B["theta"]).max()),
                theta_mean_abs_diff=float(np.abs(A["theta"] - B["theta"]).mean()),
                theta_doc_argmax_agree=float((A["theta"].argmax(1) == B["theta"].argmax(1)).mean()),
                phi_max_abs_diff=float(np.abs(A["phi"] - B["phi"]).max()),
                score_spearman=_spearman(A["score"], B["score"]),
                lowest_0p1pct_overlap=_topk_overlap(A["score"], B["score"], k_top),
                lowest_0p5pct_overlap=_topk_overlap(A["score"], B["score"], 5 * k_top),
                lowest_1pct_overlap=_topk_overlap(A["score"], B["score"], 10 * k_top),
            )
            tc, na, nb = _tie_closed_overlap(A["score"], B["score"], k_top)
            out["pairs"][f"{a} vs {b}"].update(lowest_0p1pct_tie_closed_overlap=tc, tie_closed_set_sizes=f"{na}/{nb}",
                                               distinct_scores_in_lowest_0p1pct=int(np.unique(
                                                   np.sort(A["score"], kind="stable")[:k_top]).size))
    print(json.dumps(dict(engines={k: {kk: vv for kk, vv in v.items() if kk != "likelihood_trajectory"}
                                   for k, v in out["engines"].items()}, pairs=out["pairs"]), indent=1), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    if args.md:
        ecols = ["seconds", "em_iterations", "final_likelihood", "alpha"]
        pcols = list(next(iter(out["pairs"].values())).keys()) if out["pairs"] else []
        fmt = lambda v: f"{v:.6g}" if isinstance(v, float) else str(v)
        src = "DNS" if args.corpus == "dns" else "netflow"
        sub = f", sub-sampled to the {args.keep_longest} longest + random documents" if args.sub_nnz else ""
        lines = ["# Precision / schedule parity: GPU engines vs lda-c (literal per-word Gauss-Seidel, fp64)", "",
                 f"Corpus: synthetic 1-day {src} ({args.events} events, seed {args.seed}{sub}), longest document "
                 f"{int(corpus.lengths().max())} words (block schedule chunk {-(-int(corpus.lengths().max()) // GS_U)} "
                 f"words at U = {GS_U}): "
                 f"{corpus.num_docs} docs, {corpus.num_terms} words, {len(corpus.word_idx)} entries; "
                 f"K = {args.topics}, lda-c default settings, same random init (seed {args.seed}). "
                 f"Scores = theta_d . phi_w over every corpus entry; overlap = shared fraction of the "
                 f"{k_top} lowest-scoring (most suspicious) entries.", "",
                 "| engine | " + " | ".join(ecols) + " |", "|---" * (len(ecols) + 1) + "|"]
        lines += [f"| {n} | " + " | ".join(fmt(e[c]) for c in ecols) + " |" for n, e in out["engines"].items()]
        lines += ["", "| pair | " + " | ".join(pcols) + " |", "|---" * (len(pcols) + 1) + "|"]
        lines += [f"| {n} | " + " | ".join(fmt(e[c]) for c in pcols) + " |" for n, e in out["pairs"].items()]
        with open(args.md, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
