"""ECDF quantile cuts and binning (reference: flow_pre_lda.scala:102-143, dns_pre_lda.scala:234-275;
SURVEY.md C4c, hot ops H9/H10).

The reference computes, per column,

    F(v)  = #{x <= v} / N                          (compute_ecdf: reduceByKey + sortByKey + prefix sums)
    cut_q = max({0} U {v : F(v) < q})              (distributed_quantiles: aggregate with max, init 0)
    bin   = #{cut : value > cut}                   (bin_column)

Here the same rule runs as one sort + segmented prefix sum on the device.  Rows
can carry integer weights (the analyst-feedback rows are duplicated DUPFACTOR
times in the reference, flow_pre_lda.scala:262; weights give identical counts
without materialising copies).  F is formed exactly like the JVM does: an
exact integer cumulative count divided by N in double precision.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

DECILES = (0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9)
QUINTILES = (0.0, 0.2, 0.4, 0.6, 0.8)


def ecdf_cuts(values: torch.Tensor, quantiles: Sequence[float], weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Cuts for `quantiles` from a 1-D float64 tensor (any device). Returns float64 [len(quantiles)]."""
    v = values.to(torch.float64).reshape(-1)
    q = torch.tensor(list(quantiles), dtype=torch.float64, device=v.device)
    if v.numel() == 0:
        return torch.zeros_like(q)
    if weights is None:
        uniq, counts = torch.unique(v, sorted=True, return_counts=True)
        counts = counts.to(torch.int64)
    else:
        w = weights.to(device=v.device, dtype=torch.int64).reshape(-1)
        uniq, inv = torch.unique(v, sorted=True, return_inverse=True)
        counts = torch.zeros(uniq.numel(), dtype=torch.int64, device=v.device).index_add_(0, inv, w)
    cum = torch.cumsum(counts, 0)
    F = cum.to(torch.float64) / cum[-1].to(torch.float64)
    # largest index with F < q  (F is non-decreasing)
    idx = torch.searchsorted(F, q, right=False) - 1
    cand = torch.where(idx >= 0, uniq[idx.clamp_min(0)], torch.zeros_like(q))
    return torch.maximum(cand, torch.zeros_like(q))


def ecdf_cuts_reference(values, quantiles, weights=None) -> np.ndarray:
    """Literal (slow) transcription of compute_ecdf + distributed_quantiles for tests."""
    vals = np.asarray(values, dtype=np.float64)
    w = np.ones(vals.size, np.int64) if weights is None else np.asarray(weights, np.int64)
    counts = {}
    for x, c in zip(vals.tolist(), w.tolist()):
        counts[x] = counts.get(x, 0) + c
    keys = sorted(counts)
    N = float(sum(counts.values()))
    run = 0.0
    ecdf = []
    for k in keys:
        run = run + counts[k]
        ecdf.append((k, run / N))
    acc = [0.0] * len(quantiles)
    for k, F in ecdf:
        for i, q in enumerate(quantiles):
            if F < q:
                acc[i] = max(acc[i], k)
    return np.asarray(acc)


def bin_values(values: torch.Tensor, cuts: torch.Tensor) -> torch.Tensor:
    """bin = #{cut : value > cut} (int64).  Cuts need not be sorted."""
    c = cuts.to(values.device, torch.float64)
    return (values.to(torch.float64).unsqueeze(-1) > c).sum(-1)


def format_cuts(cuts) -> str:
    """Space-separated cuts as the reference prints them (println(cuts.mkString(",")) uses ','; the
    legacy flow_qtiles file uses ' ' inside a group)."""
    from ..io.javafmt import java_double
    return " ".join(java_double(float(c)) for c in cuts)


def parse_qtiles(text: str):
    """Legacy `flow_qtiles` format (qtiles.py / gen_qtiles.sh): "byte cuts,pkt cuts,time cuts",
    each a space-separated list starting with 0."""
    groups = [g.split() for g in text.strip().split(",")]
    if len(groups) != 3:
        raise ValueError("flow_qtiles needs three comma-separated groups (ibyt, ipkt, time)")
    return {name: np.asarray([float(x) for x in g], np.float64) for name, g in zip(("ibyt", "ipkt", "time"), groups)}


def dump_qtiles(ibyt, ipkt, time) -> str:
    def fmt(a):
        out = []
        for x in a:
            x = float(x)
            out.append(str(int(x)) if x.is_integer() else repr(x))
        return " ".join(out)
    return ",".join(fmt(a) for a in (ibyt, ipkt, time))
