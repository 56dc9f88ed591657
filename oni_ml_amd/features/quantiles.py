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

from .quantile_levels import DECILES, QUINTILES  # noqa: F401  (re-exported)


def ecdf_cuts(values: torch.Tensor, quantiles: Sequence[float], weights: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Cuts for `quantiles` from a 1-D float64 tensor (any device). Returns float64 [len(quantiles)]."""
    v = values.to(torch.float64).reshape(-1)
    q = torch.tensor(list(quantiles), dtype=torch.float64, device=v.device)
    if v.numel() == 0:
        return torch.zeros_like(q)
    from ..ops import sortgroup as SG
    if weights is None:
        uniq, counts = SG.unique(v, return_counts=True)
    else:
        uniq, counts = SG.segment_sums(v, weights.to(device=v.device, dtype=torch.int64).reshape(-1))
    return ecdf_cuts_from_hist(uniq, counts, quantiles)


def ecdf_cuts_from_hist(uniq: torch.Tensor, counts: torch.Tensor, quantiles: Sequence[float]) -> torch.Tensor:
    """The cut rule on a weighted histogram (sorted distinct values, integer weights): the form the
    row-sharded featurization merges per-rank histograms into (features/flow_dist.py)."""
    q = torch.tensor(list(quantiles), dtype=torch.float64, device=uniq.device)
    if uniq.numel() == 0:
        return torch.zeros_like(q)
    counts = counts.to(torch.int64)
    cum = torch.cumsum(counts, 0)
    F = cum.to(torch.float64) / cum[-1].to(torch.float64)
    # largest index with F < q  (F is non-decreasing)
    idx = torch.searchsorted(F, q, right=False) - 1
    cand = torch.where(idx >= 0, uniq.index_select(0, idx.clamp_min(0)), torch.zeros_like(q))
    # max(cand, 0) as a select: torch.maximum's first call costs a cold process 120 ms (ops/sortgroup.py);
    # the same bits (+0.0 for cand <= 0, -0.0 included; cand is never NaN: F(NaN) = 1 >= q)
    return torch.where(cand > 0, cand, torch.zeros_like(q))


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


# ---------------------------------------------------------------------------
# gen_qtiles.sh + qtiles.py (reference gen_qtiles.sh:9-19, qtiles.py:9-21)
# ---------------------------------------------------------------------------
def hive_ntile_max(values, n: int, order_key=None):
    """``SELECT max(v), qtile FROM (SELECT v, ntile(n) OVER (ORDER BY key) AS qtile ...) GROUP BY qtile``.

    Hive's ntile puts rows (ordered by ``order_key``, default the values) into n buckets whose
    sizes differ by at most one, the first N mod n buckets holding the extra row; with fewer
    rows than buckets every row is its own bucket.  Returns [(max, tile)] in tile order."""
    v = np.asarray(values, np.float64)
    key = v if order_key is None else np.asarray(order_key)
    N = v.size
    if N == 0:
        return []
    order = np.lexsort(key.T[::-1]) if key.ndim == 2 else np.argsort(key, kind="stable")
    vs = v[order]
    tiles = min(n, N)
    base, extra = divmod(N, tiles)
    out, start = [], 0
    for t in range(tiles):
        size = base + (1 if t < extra else 0)
        out.append((float(vs[start:start + size].max()), t + 1))
        start += size
    return out


def _hive_num(x: float, integral: bool) -> str:
    """Hive CLI rendering: bigint columns as integers, double columns as Java Double.toString."""
    from ..io.javafmt import java_double
    return str(int(x)) if integral else java_double(x)


def gen_qtiles_tsv(ibyt, ipkt, hour, minute) -> str:
    """qtiles.tsv of gen_qtiles.sh: ibyt deciles, ipkt ntile(3), time deciles over (hour, minute),
    one ``max<TAB>qtile`` line per tile; a ``|`` line separates the three queries (the separator
    qtiles.py splits groups on)."""
    hour = np.asarray(hour, np.float64)
    minute = np.asarray(minute, np.float64)
    dectime = hour + minute / 60.0
    groups = [
        [(_hive_num(m, True), t) for m, t in hive_ntile_max(ibyt, 10)],
        [(_hive_num(m, True), t) for m, t in hive_ntile_max(ipkt, 3)],
        [(_hive_num(m, False), t) for m, t in hive_ntile_max(dectime, 10, np.stack([hour, minute], 1))],
    ]
    lines = []
    for gi, g in enumerate(groups):
        if gi:
            lines.append("|")
        lines.extend(f"{m}\t{t}" for m, t in g)
    return "\n".join(lines) + "\n"


def qtiles_from_tsv(tsv: str) -> str:
    """qtiles.py: "0 " then each first column + " "; a "|" row closes the group with ",0 "."""
    import csv
    import io
    out = "0 "
    for row in csv.reader(io.StringIO(tsv), delimiter="\t", quotechar='"'):
        if not row:
            continue
        if row[0] == "|":
            out = out[:-1]
            out += ",0 "
        else:
            out += "%s " % (row[0])
    return out
