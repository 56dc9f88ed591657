"""Event scoring + threshold + rank (reference: flow_post_lda.scala:227-248, dns_post_lda.scala:312-331;
SURVEY.md C5c/C5d/C7c/C7d, hot ops H12/H13).

    score(doc, word) = sum_{k<K} θ[doc]_k * φ[word]_k      (unknown doc/word -> constant default vector)
    flow key         = min(score(sip, src_word), score(dip, dest_word))
    output           = rows with key < TOL, ascending by key (sortByKey)

The gather-dot runs in the fused HIP kernel `score_events` (strict IEEE f64,
sequential over topics, as the JVM evaluates it); the survivors are compacted
and sorted on the device; only the flagged rows travel back to the host.
Ties keep input order (stable sort; Spark's order for equal keys is unspecified).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch


@dataclass
class TopicModel:
    """θ / φ tables on the device plus the name -> row lookups the scorers use."""
    theta: torch.Tensor            # [D, K] f64
    phi: torch.Tensor              # [V, K] f64
    K: int
    default: float                 # default-vector value for misses

    @staticmethod
    def build(theta: np.ndarray, phi: np.ndarray, default: float, device, K: Optional[int] = None) -> "TopicModel":
        K = int(theta.shape[1] if K is None else K)
        th = torch.from_numpy(np.ascontiguousarray(theta[:, :K], np.float64)).to(device)
        ph = torch.from_numpy(np.ascontiguousarray(phi[:, :K], np.float64)).to(device)
        return TopicModel(th, ph, K, float(default))


def default_value(source: str, K: int, strict: bool) -> float:
    """Miss vector: flow 0.05 x 20, dns 0.1 x 20 in the reference (sums 1.0 and 2.0); 1/K when fixed."""
    if strict:
        return 0.05 if source == "flow" else 0.1
    return 1.0 / K


def score(model: TopicModel, doc_a, word_a, doc_b=None, word_b=None, tol: float = float("inf")):
    """Returns (score_a, score_b|None, key, flag) device tensors."""
    dev = model.theta.device
    if dev.type == "cuda":
        from ..ops import hip as H
        return H.score_events(model.theta, model.phi, model.K, model.default, doc_a.to(torch.int32).contiguous(),
                              word_a.to(torch.int32).contiguous(),
                              None if doc_b is None else doc_b.to(torch.int32).contiguous(),
                              None if word_b is None else word_b.to(torch.int32).contiguous(), tol)
    from ..ops.reference import score as ref
    return ref(model.theta, model.phi, model.K, model.default, doc_a, word_a, doc_b, word_b, tol)


def key_quantiles(key: torch.Tensor, qs=(1e-4, 1e-3, 1e-2, 0.1, 0.5), sample: int = 1 << 18) -> dict:
    """Quantiles of the events' scores (a strided sample of at most ``sample``), for choosing TOL: the
    fraction q of events scoring below key_q<q> would be flagged.  Metrics only: the sample goes to the
    host (a first torch.quantile on the device cost 57 ms of a cold process's wall)."""
    n = key.numel()
    if n == 0:
        return {}
    k = key[:: max(1, -(-n // sample))].to(torch.float64).cpu().numpy()
    v = np.quantile(k, np.asarray(qs, np.float64))
    return {f"key_q{q:g}": float(x) for q, x in zip(qs, v)}


def rank_flagged(key: torch.Tensor, flag: torch.Tensor) -> torch.Tensor:
    """Indices of flagged rows in ascending key order (stable) as an int64 host array."""
    from ..ops import sortgroup as SG
    sel, _ = SG.compact(torch.arange(flag.numel(), device=flag.device), flag.reshape(-1).to(torch.bool))
    if sel.numel() == 0:
        return np.zeros(0, np.int64)
    order = SG.sort_stable(SG.gather(key, sel))[1]
    return SG.gather(sel, order).cpu().numpy().astype(np.int64)


def lookup_sorted(keys_sorted: torch.Tensor, values_idx: torch.Tensor, query: torch.Tensor) -> torch.Tensor:
    """Map query keys through a sorted key table -> row index (or -1)."""
    if keys_sorted.numel() == 0:
        return torch.full_like(query, -1, dtype=torch.int64)
    i = torch.searchsorted(keys_sorted, query).clamp_max(keys_sorted.numel() - 1)
    hit = keys_sorted[i] == query
    return torch.where(hit, values_idx[i], torch.full_like(i, -1))


class KeyIndex:
    """word-key -> word-row lookup (device).  `valid` masks rows the reference could never match
    (strict mode: word names longer than 20 bytes are truncated in word_results.csv)."""

    def __init__(self, keys: np.ndarray, device, valid: Optional[np.ndarray] = None):
        keys = np.asarray(keys, np.int64)
        rows = np.arange(keys.size, dtype=np.int64)
        if valid is not None:
            keys, rows = keys[valid], rows[valid]
        o = np.argsort(keys, kind="stable")
        self.keys = torch.from_numpy(keys[o]).to(device)
        self.rows = torch.from_numpy(rows[o]).to(device)

    def __call__(self, q: torch.Tensor) -> torch.Tensor:
        out = lookup_sorted(self.keys, self.rows, q.to(torch.int64))
        return torch.where(q >= 0, out, torch.full_like(out, -1))
