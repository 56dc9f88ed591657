"""Row-sharded corpus builder: every rank's (ip, word) counts -> this rank's document shard of the
lda-c corpus, without replicating doc_wc on any rank (lda_pre.py on the reference's ``cat part-*``
file, ml_ops.sh:59-67).

Steps (all tensor collectives, parallel/shardio.py):

1. route each counted line to the rank owning its document's id range (``all_to_all``) and merge
   the partial counts there: each rank now holds a contiguous block of every doc_wc section
   (doc_wc = the sections one after another, each sorted by (ip id, word key));
2. a line's global position in doc_wc = section base + lines of lower ranks + local index;
3. word ids (words.dat, 0-based): first appearance = the minimum position of each word -- per-rank
   minima all-gathered and merged (V rows, not nnz);
4. doc ids (doc.dat, 1-based): a document's first line decides its place, and the blocks are in
   (section, rank) order, so a document's id is its block's offset plus its rank inside the block;
5. the engine shards (``parallel.dist.engine_bounds`` of the global doc_ptr: chain-aware by default)
   from every document's length, gathered as (id, length) pairs; the entries move to the rank owning
   their document (``all_to_all``), where they become this rank's CSR shard.

The result -- shard bounds, every entry's word id, every document's id and entries in line order --
is identical to ``corpus.builder.lda_pre`` of the whole doc_wc (tests/test_sharded_pipeline.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np
import torch

from ..parallel import shardio as SIO
from .builder import DocWordCounts, concat, count_pairs
from .csr import Corpus

_I64MAX = np.iinfo(np.int64).max


@dataclass
class ShardedCorpus:
    corpus: Corpus                  # this rank's documents [d0, d1): local doc ids, global word ids
    doc_range: Tuple[int, int]
    doc_keys: np.ndarray            # [d1 - d0] ip ids (global dictionary) of this shard's documents
    num_docs: int                   # global D
    nnz: int                        # global nnz
    word_keys: np.ndarray           # [V] word key of every word id (words.dat order), on every rank
    bounds: List[int]               # engine shard bounds [0, ..., D]
    lines: List[DocWordCounts]      # this rank's block of every doc_wc section (doc_wc.dat)


def _route(ctx, sec: DocWordCounts, n_ids: int, device) -> DocWordCounts:
    """Lines of every rank -> the rank owning doc ids [n_ids r / N, n_ids (r + 1) / N), counts merged."""
    N = SIO.world(ctx)
    doc = sec.doc.to(torch.int64).cpu()
    if N == 1:
        return sec
    owner = (doc * N) // max(int(n_ids), 1)
    splits = torch.bincount(owner, minlength=N).tolist()
    packed = torch.stack([doc, sec.word.to(torch.int64).cpu(), sec.count.to(torch.int64).cpu()], 1).numpy()
    # lines are sorted by doc id, so each owner's lines are one contiguous run
    cuts = np.concatenate([[0], np.cumsum(splits)])
    recv = SIO.alltoallv(ctx, [packed[cuts[s]:cuts[s + 1]] for s in range(N)])
    allp = torch.from_numpy(np.concatenate(recv)).to(device)
    if allp.numel() == 0:
        e = torch.zeros(0, dtype=torch.int64, device=device)
        return DocWordCounts(e, e, e)
    return count_pairs(allp[:, 0], allp[:, 1], allp[:, 2])


def build_sharded(ctx, sections: Sequence[DocWordCounts], n_ids: int, merge: bool = False,
                  device="cpu", K: int = None) -> ShardedCorpus:
    """``sections``: this rank's (global ip id, word key, count) lines per doc_wc section, each sorted by
    (ip, word) with counts merged (``count_pairs``); ``n_ids``: size of the global ip dictionary;
    ``merge``: sum a (doc, word) pair's counts across sections (compat=fixed, ``concat(merge=True)``)."""
    device = torch.device(device)
    N, r = SIO.world(ctx), SIO.rank(ctx)
    owned = [_route(ctx, s, n_ids, device) for s in sections]
    if merge and len(owned) > 1:
        owned = [concat(owned, merge=True)]
    S = len(owned)
    # ---- global line positions
    ns = np.asarray([o.n for o in owned], np.int64)
    allns = np.stack(SIO.allgather_array(ctx, ns))                       # [N, S]
    sec_base = np.concatenate([[0], np.cumsum(allns.sum(0))])[:S]
    my_base = sec_base + allns[:r].sum(0)
    docs = torch.cat([o.doc.to(torch.int64) for o in owned]).cpu()
    words = torch.cat([o.word.to(torch.int64) for o in owned]).cpu()
    counts = torch.cat([o.count.to(torch.int64) for o in owned]).cpu()
    pos = torch.cat([torch.arange(int(n), dtype=torch.int64) + int(b) for n, b in zip(ns, my_base)]) \
        if ns.sum() else torch.zeros(0, dtype=torch.int64)
    nl = int(pos.numel())
    if int(allns.sum()) == 0:
        raise ValueError("empty doc_wc: no (ip, word) pairs survived featurization")
    # ---- words.dat: first appearance over the whole doc_wc
    uw, winv = torch.unique(words, return_inverse=True)
    wmin = torch.full((uw.numel(),), _I64MAX, dtype=torch.int64).scatter_reduce_(0, winv, pos, reduce="amin")
    gw_parts = SIO.allgather_array(ctx, uw.numpy())
    gm_parts = SIO.allgather_array(ctx, wmin.numpy())
    gw, ginv = torch.unique(torch.from_numpy(np.concatenate(gw_parts)), return_inverse=True)
    gmin = torch.full((gw.numel(),), _I64MAX, dtype=torch.int64).scatter_reduce_(
        0, ginv, torch.from_numpy(np.concatenate(gm_parts)), reduce="amin")
    worder = torch.argsort(gmin)
    wid_of_sorted = torch.empty_like(worder)
    wid_of_sorted[worder] = torch.arange(worder.numel())
    word_keys = gw[worder].numpy()
    wid = wid_of_sorted[torch.searchsorted(gw, words)] if nl else torch.zeros(0, dtype=torch.int64)
    # ---- doc.dat: a document's place is its first line's; blocks in (section, rank) order
    ud, dinv = torch.unique(docs, return_inverse=True)
    dfirst = torch.full((ud.numel(),), _I64MAX, dtype=torch.int64).scatter_reduce_(0, dinv, pos, reduce="amin")
    fsec = torch.searchsorted(torch.from_numpy(sec_base[1:].copy()), dfirst, right=True) if S > 1 \
        else torch.zeros_like(dfirst)
    dorder = torch.argsort(dfirst)                                        # (section, position) order
    F = torch.bincount(fsec, minlength=S).numpy().astype(np.int64)
    allF = np.stack(SIO.allgather_array(ctx, F))                          # [N, S]
    blk_off = np.concatenate([[0], np.cumsum(allF.T.reshape(-1))])[:-1].reshape(S, N)   # block (s, r)
    D = int(allF.sum())
    fs_sorted = fsec[dorder]
    start_in_sorted = torch.from_numpy(np.concatenate([[0], np.cumsum(F)])[:-1].copy())
    k = torch.arange(dorder.numel(), dtype=torch.int64)
    idx_sorted = torch.from_numpy(blk_off[:, r].copy())[fs_sorted] + (k - start_in_sorted[fs_sorted])
    doc_index = torch.empty_like(idx_sorted)
    doc_index[dorder] = idx_sorted                                        # per unique local doc
    # ---- global doc_ptr of this rank's documents, from per-block nnz totals
    dlen = torch.bincount(dinv, minlength=ud.numel()).to(torch.int64)
    len_sorted = dlen[dorder]
    B = np.zeros(S, np.int64)
    np.add.at(B, fs_sorted.numpy(), len_sorted.numpy())
    allB = np.stack(SIO.allgather_array(ctx, B))                          # [N, S]
    nnz = int(allB.sum())
    blk_nnz_off = np.concatenate([[0], np.cumsum(allB.T.reshape(-1))])[:-1].reshape(S, N)
    cum_in_sorted = torch.cumsum(len_sorted, 0) - len_sorted               # exclusive, over my sorted docs
    cum_sec_start = torch.from_numpy(np.concatenate([[0], np.cumsum(B)])[:-1].copy())
    start_sorted = torch.from_numpy(blk_nnz_off[:, r].copy())[fs_sorted] + (cum_in_sorted - cum_sec_start[fs_sorted])
    # ---- engine shard bounds (parallel.dist.engine_bounds of the global doc_ptr): every rank's
    # (document id, length) pairs gathered, so every rank builds the same global doc_ptr (D lengths,
    # 16 bytes per document) and applies the engine's own rule -- chain-aware by default
    bounds = [0, D]
    if N > 1:
        from ..parallel.dist import engine_bounds
        pairs = np.stack([idx_sorted.numpy(), len_sorted.numpy()], 1) if idx_sorted.numel() else \
            np.zeros((0, 2), np.int64)
        allp = np.concatenate(SIO.allgather_array(ctx, pairs))
        glen = np.zeros(D, np.int64)
        glen[allp[:, 0]] = allp[:, 1]
        gptr = np.concatenate([[0], np.cumsum(glen)])
        cut = engine_bounds(gptr, N, K)
        bounds = [0] + [int(b1) for _, b1 in cut]
    # ---- entries to the shard owners: (doc index, word id, count, ip id), line order kept per doc
    line_doc = doc_index[dinv]
    order = torch.sort(line_doc, stable=True).indices
    ent = torch.stack([line_doc[order], wid[order], counts[order], docs[order]], 1).numpy() if nl \
        else np.zeros((0, 4), np.int64)
    dest = np.searchsorted(np.asarray(bounds[1:-1], np.int64), ent[:, 0], side="right")
    cuts = np.searchsorted(dest, np.arange(N + 1), side="left")
    recv = SIO.alltoallv(ctx, [ent[cuts[s]:cuts[s + 1]] for s in range(N)]) if N > 1 else [ent]
    allent = np.concatenate(recv) if recv else np.zeros((0, 4), np.int64)
    # each document's entries come from one rank, already in line order: a stable sort by doc index
    o = np.argsort(allent[:, 0], kind="stable")
    allent = allent[o]
    d0, d1 = bounds[r], bounds[r + 1]
    rel = allent[:, 0] - d0
    ptr = np.searchsorted(rel, np.arange(d1 - d0 + 1), side="left").astype(np.int64)
    first = ptr[:-1]
    doc_keys = allent[first, 3] if d1 > d0 else np.zeros(0, np.int64)
    corpus = Corpus(ptr, allent[:, 1].astype(np.int32), allent[:, 2], int(word_keys.size))
    return ShardedCorpus(corpus=corpus, doc_range=(d0, d1), doc_keys=doc_keys, num_docs=D, nnz=nnz,
                         word_keys=word_keys, bounds=bounds, lines=owned)
