"""The ECDF cut rule of features/quantiles.py on the host, without torch (numpy only): the DNS prefetch
child computes dns_pre's and dns_post's cuts while the parent imports torch (pipeline/prefetch.py).

Same arithmetic as ``quantiles.ecdf_cuts``: sorted distinct values with exact integer (weighted)
counts, F = cumulative count / total in double, cut_q = max({0} U {v : F(v) < q}) -- identical bits.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np


def ecdf_cuts_np(values: np.ndarray, quantiles: Sequence[float], weights: Optional[np.ndarray] = None) -> np.ndarray:
    v = np.asarray(values, np.float64).reshape(-1)
    q = np.asarray(list(quantiles), np.float64)
    if v.size == 0:
        return np.zeros_like(q)
    uniq, inv = np.unique(v, return_inverse=True)
    if weights is None:
        counts = np.bincount(inv, minlength=uniq.size).astype(np.int64)
    else:
        # integer weights: an exact sum per distinct value (bincount's float64 sum is exact while the day's
        # total stays below 2^53; np.add.at, exact everywhere, takes ~10x longer)
        w = np.asarray(weights, np.int64).reshape(-1)
        if int(w.sum()) < (1 << 53):
            counts = np.bincount(inv.reshape(-1), weights=w, minlength=uniq.size).astype(np.int64)
        else:
            counts = np.zeros(uniq.size, np.int64)
            np.add.at(counts, inv, w)
    cum = np.cumsum(counts)
    F = cum.astype(np.float64) / np.float64(cum[-1])
    idx = np.searchsorted(F, q, side="left") - 1
    cand = np.where(idx >= 0, uniq[np.clip(idx, 0, None)], 0.0)
    return np.where(cand > 0, cand, 0.0)     # max(cand, 0) as quantiles.ecdf_cuts takes it (-0.0 -> +0.0)


# dns_pre_lda.scala's cuts: deciles of unix_tstamp and frame_len over every row, quintiles of the subdomain
# length, entropy and label count over the rows with a value > 0 (features/dns.py featurize)
DNS_CUT_COLUMNS = (("unix_tstamp", "deciles", False), ("frame_len", "deciles", False),
                   ("subdomain_length", "quintiles", True), ("entropy", "quintiles", True),
                   ("num_periods", "quintiles", True))


def dns_cuts_np(values: dict, weight: np.ndarray, n: int, threads: int = 8) -> dict:
    """{column: cuts} over the first n rows: the five columns on threads, each through the native
    ``ecdf_cuts_cols`` (no GIL; bitwise ecdf_cuts_np, which took ~0.15 s a column at 2 M rows)."""
    from concurrent.futures import ThreadPoolExecutor
    from .quantile_levels import DECILES, QUINTILES
    from ..ops import native
    w = np.asarray(weight[:n], np.int64)

    def one(spec):
        name, levels, positive = spec
        v = np.asarray(values[name][:n], np.float64)
        q = list(DECILES if levels == "deciles" else QUINTILES)
        vv, ww = (v[v > 0], w[v > 0]) if positive else (v, w)
        return name, np.asarray(native.lib().ecdf_cuts_cols([vv], ww, [q])[0], np.float64)

    with ThreadPoolExecutor(max(1, min(threads, len(DNS_CUT_COLUMNS)))) as ex:
        return dict(ex.map(one, DNS_CUT_COLUMNS))


def flow_cuts_np(table, n: int) -> dict:
    """flow_pre's cuts of the first ``n`` rows of a flow TextTable (features/flow.py featurize): deciles of
    the time column (hour + minute / 60) + second / 3600 and of ibyt, quintiles of ipkt, weighted by the rows'
    weights -- the same rule and bits as the device ``ecdf_cuts``."""
    from .flow_io import C_HOUR, C_IBYT, C_IPKT, C_MIN, C_SEC
    from .quantile_levels import DECILES, QUINTILES
    from ..ops import native
    w = np.asarray(table.weights()[:n], np.int64)
    col = lambda c: np.asarray(table.numeric(c)[:n], np.float64)
    time = (col(C_HOUR) + col(C_MIN) / 60) + col(C_SEC) / 3600
    # the three columns on native threads without the GIL (ecdf_cuts_np's numpy unique slowed the torch
    # import running beside it); ecdf_cuts_np is the test oracle
    c = native.lib().ecdf_cuts_cols([time, col(C_IBYT), col(C_IPKT)], w, [list(DECILES), list(DECILES),
                                                                       list(QUINTILES)])
    return dict(time=np.asarray(c[0], np.float64), ibyt=np.asarray(c[1], np.float64),
                ipkt=np.asarray(c[2], np.float64))
