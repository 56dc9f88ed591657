#!/usr/bin/env python
"""Strong-scaling ceiling of document data parallelism, measured on one GPU.

oni-lda-c splits one model.dat over its MPI ranks (ml_ops.sh:22-23,80); the engine shards the
documents contiguously and nnz-balanced (parallel/dist.py shard_bounds).  An N-GPU EM iteration
takes max over ranks r of (rank r's E-step + M-step on its shard) + the class_word reduction.  This
script measures the first term exactly, one shard at a time on one GPU, and models the second:

  1. train the whole corpus a few EM iterations (the global model of a real run);
  2. for N = 1, 2, 4, 8 and every rank r: an engine on shard r alone (global vocabulary), started
     from that global model, times one EM iteration (median of --reps, the model reloaded before
     each) -- the work rank r does per iteration of the N-GPU run;
  3. the longest document alone: the chain floor no document sharding can go below;
  4. the dense class_word all-reduce (K V 8 bytes): a ring over the xGMI links (2 (N-1)/N bytes per
     153 GB/s link) and the fully connected mesh's direct all-to-all form (2 bytes / (N 153 GB/s)),
     each + 10 us per step of latency.

  python scripts/strong_emulated.py --configs headline,k50,dns,c5shard --json out.json --md out.md
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "headline": dict(kind="flow", events=1_000_000, K=20, label="config 2: flow 1-day, K=20"),
    "k50": dict(kind="flow", events=1_000_000, K=50, label="config 3: flow 1-day, K=50"),
    "dns": dict(kind="dns", events=2_000_000, K=20, label="config 4: DNS 1-day, K=20"),
    "c5shard": dict(kind="flow", events=12_500_000, K=100, label="config 5 shard: flow 12.5M events, K=100"),
    # BASELINE config 5 itself: the month's real corpus, cut into the N ranks' shards
    "c5": dict(kind="flow", events=100_000_000, days=30, K=100, warm_em=3, reps=3,
               label="config 5: flow 30-day month (100M events), K=100"),
}
LINK_BPS = 153e9
STEP_LAT = 10e-6


def _corpus(cfg):
    if cfg["kind"] == "dns":
        from oni_ml_amd.pipeline.dns import synthetic_dns_corpus
        c, _ = synthetic_dns_corpus(events=cfg["events"], seed=0, device="cuda")
    else:
        from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
        days = cfg.get("days", 1)
        c, _ = synthetic_flow_corpus(events=cfg["events"], seed=0, device="cuda", threads=16,
                                     chunk_events=-(-cfg["events"] // days) if days > 1 else 0)
    return c


def _exchange_model(c, bounds, K):
    """The engine's sparse class_word exchange (parallel/dist.py VocabExchange) for these shards: rows
    rank r sends = sum over s != r of |words(r) & words(s)|; an all_to_all over the fully connected
    mesh moves a rank's rows over its N - 1 links at once.  Returns (max rows sent, ms, dense ms)."""
    from oni_ml_amd.ops import hip as H
    KS = H.padded_topics(K)
    sets = [np.unique(c.word_idx[c.doc_ptr[d0]:c.doc_ptr[d1]]) for d0, d1 in bounds]
    N = len(bounds)
    cnt = np.zeros(c.num_terms, np.int32)
    for w in sets:
        cnt[w] += 1
    rows = [int((cnt[w] - 1).sum()) for w in sets]     # each local word shared with cnt - 1 other ranks
    mx = max(rows)
    t = mx * KS * 8 / ((N - 1) * LINK_BPS) + STEP_LAT
    dense = 2 * KS * 8 * c.num_terms / (N * LINK_BPS) + 2 * STEP_LAT
    return mx, t, dense


def _local(sh, V, lb, compact):
    """(corpus, model) of one rank's documents: with ``compact`` the vocabulary is the shard's own words
    (renumbered, beta columns sliced), as a rank's real iteration touches them -- the sparse exchange
    engine's M-step and suff-stats cover only its local rows (parallel/dist.py VocabExchange, em.py
    _overlap); without, a full-V M-step per rank (~4.5 ms at config 5) is charged to every shard."""
    from oni_ml_amd.corpus.csr import Corpus
    if not compact:
        return Corpus(sh.doc_ptr, sh.word_idx, sh.counts, V), lb
    words, inv = np.unique(sh.word_idx, return_inverse=True)
    return Corpus(sh.doc_ptr, inv.astype(np.int32), sh.counts, int(words.size)), np.ascontiguousarray(lb[:, words])


def _time_iteration(eng, lb, alpha, vmi, D, reps):
    ts = []
    for _ in range(reps):
        eng.init_from_model(lb, alpha)
        eng.var_max_iter = vmi
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.em_iterations(1, True, D, stop=False)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="headline,k50,dns,c5shard")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--warm-em", type=int, default=6)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--compact", type=int, default=1,
                    help="1: each shard on its own words (the sparse-exchange engine's local M-step); 0: full V")
    ap.add_argument("--json")
    ap.add_argument("--md")
    a = ap.parse_args()
    t_start = time.perf_counter()

    def heartbeat():     # config 5's corpus build prints nothing for minutes otherwise
        while True:
            time.sleep(60)
            print(json.dumps(dict(heartbeat_s=round(time.perf_counter() - t_start))), flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    from oni_ml_amd.corpus.csr import Corpus
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.parallel.dist import shard_bounds
    out = {}
    for name in a.configs.split(","):
        cfg = CONFIGS[name]
        c = _corpus(cfg)
        K, D = cfg["K"], c.num_docs
        full = LDAEngine(c, K, LDASettings(), backend="hip", seed=0, precision="fp64")
        full.init_random()
        full.em_iterations(cfg.get("warm_em", a.warm_em), True, D, stop=False)
        torch.cuda.synchronize()
        lb, alpha, vmi = full.log_beta(), full.alpha, full.var_max_iter
        reps = cfg.get("reps", a.reps)
        t_full = _time_iteration(full, lb, alpha, vmi, D, reps)
        del full
        torch.cuda.empty_cache()
        lens = c.lengths()
        dl = int(np.argmax(lens))
        one = c.slice_docs(dl, dl + 1)
        c1, lb1 = _local(one, c.num_terms, lb, a.compact)
        e1 = LDAEngine(c1, K, LDASettings(), backend="hip", seed=0, precision="fp64", local_shard=True)
        t_chain = _time_iteration(e1, lb1, alpha, vmi, D, reps)
        del e1
        rec = dict(label=cfg["label"], docs=D, nnz=c.nnz, vocab=c.num_terms, K=K, longest_doc=int(lens[dl]),
                   full_ms=round(t_full * 1e3, 4), chain_floor_ms=round(t_chain * 1e3, 4), ranks={})
        bytes_ = K * c.num_terms * 8
        for n in [int(x) for x in a.ranks.split(",")]:
            def shard_times(bounds, chains=None):
                per = []
                for d0, d1 in bounds:
                    sh = c.slice_docs(d0, d1)
                    cs_, lbs = _local(sh, c.num_terms, lb, a.compact)
                    e = LDAEngine(cs_, K, LDASettings(), backend="hip", seed=0, precision="fp64", local_shard=True)
                    per.append(_time_iteration(e, lbs, alpha, vmi, D, reps))
                    del e
                    torch.cuda.empty_cache()
                    if chains is not None:
                        # the shard's longest document alone: its chain, the floor of that rank
                        dl_ = d0 + int(np.argmax(lens[d0:d1]))
                        o1 = c.slice_docs(dl_, dl_ + 1)
                        co, lbo = _local(o1, c.num_terms, lb, a.compact)
                        e = LDAEngine(co, K, LDASettings(), backend="hip", seed=0, precision="fp64", local_shard=True)
                        chains.append((int(lens[dl_]), _time_iteration(e, lbo, alpha, vmi, D, reps)))
                        del e
                return per
            chains = []
            per = [t_full] if n == 1 else shard_times(shard_bounds(c.doc_ptr, n), chains)
            # chain-aware shards (parallel/dist.py chain_bounds, ONI_SHARD_CHAIN=1): the longest document alone
            cb = shard_bounds(c.doc_ptr, n, chain=True, K=K) if n > 1 else None
            per_chain = shard_times(cb) if cb is not None and cb != shard_bounds(c.doc_ptr, n) else None
            ring = 0.0 if n == 1 else 2 * (n - 1) / n * bytes_ / LINK_BPS + 2 * (n - 1) * STEP_LAT
            mesh = 0.0 if n == 1 else 2 * bytes_ / (n * LINK_BPS) + 2 * STEP_LAT
            mx = max(per)
            mc = max(per_chain) if per_chain else None
            if n > 1:
                xb = cb if cb is not None else shard_bounds(c.doc_ptr, n)
                xrows, xms, _ = _exchange_model(c, xb, K)
            else:
                xrows, xms = 0, 0.0
            # entries of each shard by document length class, and its distinct words: the data the engine's
            # cost-weighted cut is fitted to (parallel/dist.py doc_costs)
            edges = [0, 1, 4, 16, 64, 256, 1024, 2048, 8192, 1 << 40]

            def shard_stats(bounds):
                out_b, out_v = [], []
                for d0, d1 in bounds:
                    ln = lens[d0:d1]
                    out_b.append([int(ln[(ln > lo) & (ln <= hi)].sum()) for lo, hi in zip(edges[:-1], edges[1:])])
                    out_v.append(int(np.unique(c.word_idx[c.doc_ptr[d0]:c.doc_ptr[d1]]).size))
                return out_b, out_v
            buckets, vocab = shard_stats(shard_bounds(c.doc_ptr, n) if n > 1 else [(0, D)])
            cbuckets, cvocab = shard_stats(cb) if per_chain else (None, None)
            rec["ranks"][n] = dict(per_rank_ms=[round(x * 1e3, 4) for x in per], max_ms=round(mx * 1e3, 4),
                                   len_class_edges=edges[1:-1], per_rank_entries_by_len=buckets,
                                   per_rank_vocab=vocab, chain_aware_entries_by_len=cbuckets,
                                   chain_aware_vocab=cvocab,
                                   per_rank_longest_words=[w for w, _ in chains],
                                   per_rank_chain_ms=[round(t * 1e3, 4) for _, t in chains],
                                   chain_aware_per_rank_ms=None if per_chain is None else [round(x * 1e3, 4) for x in per_chain],
                                   chain_aware_max_ms=None if mc is None else round(mc * 1e3, 4),
                                   chain_aware_speedup_mesh=None if mc is None else round(t_full / (mc + mesh), 3),
                                   allreduce_ring_ms=round(ring * 1e3, 4), allreduce_mesh_ms=round(mesh * 1e3, 4),
                                   iter_ms_ring=round((mx + ring) * 1e3, 4), iter_ms_mesh=round((mx + mesh) * 1e3, 4),
                                   speedup_ring=round(t_full / (mx + ring), 3), speedup_mesh=round(t_full / (mx + mesh), 3),
                                   chain_bound_speedup=round(t_full / max(t_chain, 1e-12), 3),
                                   sparse_exchange_rows=xrows, sparse_exchange_ms=round(xms * 1e3, 4),
                                   iter_ms_sparse=round(((mc if mc is not None else mx) + xms) * 1e3, 4),
                                   speedup_sparse=round(t_full / ((mc if mc is not None else mx) + xms), 3))
            print(json.dumps(dict(config=name, n=n, **rec["ranks"][n])), flush=True)
        out[name] = rec
        del c
        torch.cuda.empty_cache()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
    if a.md:
        L = ["# Strong scaling emulated on one MI355X (per-shard EM iteration, max over ranks + modelled all-reduce)", ""]
        for name, rec in out.items():
            L.append(f"## {rec['label']}")
            L.append(f"docs {rec['docs']}, nnz {rec['nnz']}, V {rec['vocab']}; longest document {rec['longest_doc']} "
                     f"words; one GPU {rec['full_ms']} ms / EM iteration; **chain floor** (longest document alone) "
                     f"{rec['chain_floor_ms']} ms = at most {rec['full_ms'] / max(rec['chain_floor_ms'], 1e-9):.2f}x")
            L.append("")
            L.append("Per-rank longest document (words) and its chain alone (ms), plain cuts:")
            L.append("")
            for n, r in rec["ranks"].items():
                if r.get("per_rank_chain_ms"):
                    L.append(f"- N = {n}: " + ", ".join(f"{w} w / {t} ms" for w, t in zip(r["per_rank_longest_words"],
                                                                                        r["per_rank_chain_ms"])))
            L.append("")
            L.append("| N | max shard ms | per-rank ms | all-reduce ring / mesh ms | iteration ms (ring / mesh) | speedup (ring / mesh) | chain-aware: max shard ms, per-rank ms, speedup (mesh) | sparse exchange: rows, ms, iteration ms, speedup |")
            L.append("|---|---|---|---|---|---|---|---|")
            for n, r in rec["ranks"].items():
                ca = "—" if not r.get("chain_aware_max_ms") else (
                    f"{r['chain_aware_max_ms']}; {' '.join(str(x) for x in r['chain_aware_per_rank_ms'])}; "
                    f"{r['chain_aware_speedup_mesh']}")
                L.append(f"| {n} | {r['max_ms']} | {' '.join(str(x) for x in r['per_rank_ms'])} | "
                         f"{r['allreduce_ring_ms']} / {r['allreduce_mesh_ms']} | {r['iter_ms_ring']} / {r['iter_ms_mesh']} | "
                         f"{r['speedup_ring']} / {r['speedup_mesh']} | {ca} | {r.get('sparse_exchange_rows')}, "
                         f"{r.get('sparse_exchange_ms')}, {r.get('iter_ms_sparse')}, {r.get('speedup_sparse')} |")
            L.append("")
        open(a.md, "w").write("\n".join(L) + "\n")


if __name__ == "__main__":
    main()
