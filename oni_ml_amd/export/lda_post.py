"""Model export: the lda_post.py equivalent (reference lda_post.py:1-123).

* doc_results.csv  - ``ip,θ1 θ2 … θK``: θ = γ/Σγ per document (20 zeros when
  Σγ <= 0), the document name taken from doc.dat line j (lda_post.py:35-63).
* word_results.csv - ``word,p1 … pK``: per topic p(w|z) = exp(logβ)/Σ_w exp(logβ),
  transposed to one line per word (lda_post.py:70-122).

Values are Python-2 ``str(float)`` text ("%.12g"); sums run sequentially like
Python's builtin ``sum`` over numpy float64.  In ``strict`` compat mode the
inputs are first rounded through the "%5.10f" text lda-c writes (lda_post.py
reads final.gamma / final.beta back from disk), words are truncated to 20
bytes (the ``dtype="S20"`` array, lda_post.py:78-84) and K must be 20
(the hard-coded 20-column format, lda_post.py:42,115).
"""
from __future__ import annotations

import os
from typing import Sequence, Tuple

import numpy as np

from ..ops import native


def _host_threads() -> int:
    from .. import knobs
    return knobs.threads(16)


def _par(fn, n: int, min_block: int = 1 << 15):
    """fn(lo, hi) over [0, n) in blocks on a thread pool (numpy ufuncs release the GIL).  Every
    operation split this way is elementwise or per row, so the results are bitwise those of one call:
    config 5's θ / φ (5.7 M x 100 and 100 x 4.5 M) took ~10 s of numpy on one core."""
    t = min(_host_threads(), max(1, n // min_block))
    if t <= 1:
        fn(0, n)
        return
    from concurrent.futures import ThreadPoolExecutor
    cuts = [n * i // t for i in range(t + 1)]
    with ThreadPoolExecutor(t) as ex:
        list(ex.map(lambda i: fn(cuts[i], cuts[i + 1]), range(t)))


def doc_topics(gamma: np.ndarray, strict: bool = True) -> np.ndarray:
    """θ [D, K] float64 from γ [D, K]: each row over its sequential sum (lda_post.py:42-53; zeros where
    the sum is not positive).  Native, row-parallel, bitwise numpy's cumsum-and-divide."""
    g = np.ascontiguousarray(np.asarray(gamma, np.float64))
    if strict:
        g = native.lib().roundtrip_fixed10(g)
    if g.size == 0:
        return g.copy()
    return native.lib().doc_topics(g, _host_threads())


def word_topics(log_beta: np.ndarray, strict: bool = True) -> np.ndarray:
    """p(w|z) [V, K] float64 from log β [K, V]: numpy's exp (blocks on a thread pool), then each topic
    over its sequential sum, transposed (native; lda_post.py:88-96)."""
    lb = np.asarray(log_beta, np.float64)
    if strict:
        lb = native.lib().roundtrip_fixed10(np.ascontiguousarray(lb))
    K, V = lb.shape
    raw = np.empty((K, V), np.float64)

    def ex(lo, hi):
        np.exp(lb[:, lo:hi], out=raw[:, lo:hi])
    _par(ex, V)
    if raw.size == 0:
        return np.zeros((V, K), np.float64)
    return native.lib().topic_normalize_t(raw, _host_threads())


def truncate_s20(names: Sequence[str]) -> list:
    """numpy dtype 'S20' assignment: the UTF-8 bytes cut to 20 (trailing NULs dropped on read)."""
    out = []
    for n in names:
        b = n.encode("utf-8")[:20].rstrip(b"\x00")
        out.append(b.decode("utf-8", errors="ignore"))
    return out


def check_strict_k(K: int, strict: bool):
    if strict and K != 20:
        raise ValueError("compat=strict reproduces lda_post.py's hard-coded 20 topics; use compat=fixed for K != 20")


def _write_table(path, names, values, threads, read_back):
    n = len(names)
    if values.shape[0] != n:
        raise ValueError("names / value rows differ")
    vals = np.ascontiguousarray(values, np.float64)
    back = np.empty_like(vals) if read_back else None
    kw = {"threads": threads} if threads > 0 else {}     # 0: the writer's default (hardware, <= 16)
    native.lib().write_rows(path, None, [("dict", list(names), np.arange(n, dtype=np.int32)),
                                         ("py2row", vals, " ", back)], n=n, **kw)
    return back


def write_doc_results(path: str, doc_names: Sequence[str], theta: np.ndarray, threads: int = 0,
                      read_back: bool = False):
    """``read_back``: also return the values as a reader parses them from the file (the Python-2 str
    text read back with strtod) -- the scorers' view, produced by the same formatting pass."""
    return _write_table(path, doc_names, theta, threads, read_back)


def write_word_results(path: str, word_names: Sequence[str], phi: np.ndarray, threads: int = 0,
                       read_back: bool = False):
    return _write_table(path, word_names, phi, threads, read_back)


def export(doc_names, gamma, word_names, log_beta, doc_path, word_path, strict=True,
           read_back: bool = False) -> Tuple[np.ndarray, np.ndarray, list]:
    """Write both files; returns (θ, φ, word keys as written).  ``read_back``: θ / φ as the scorers
    parse them from the files (each value's own text read back, same pass as the write)."""
    check_strict_k(gamma.shape[1], strict)
    theta = doc_topics(gamma, strict)
    phi = word_topics(log_beta, strict)
    wnames = truncate_s20(word_names) if strict else list(word_names)
    th_b = write_doc_results(doc_path, doc_names, theta, read_back=read_back)
    ph_b = write_word_results(word_path, wnames, phi, read_back=read_back)
    if read_back:
        return th_b, ph_b, wnames
    return theta, phi, wnames


def export_deferred(doc_names, gamma, word_names, log_beta, doc_path, word_path, strict=True):
    """``export(read_back=True)`` whose two files are written on a thread: returns (θ, φ as the scorers
    parse them, word keys as written, join).  The read-back tables come from ``roundtrip_py2`` (the
    same Python-2 str -> strtod text round trip the writer's read-back performs, value by value), so
    the scoring stage starts while the files are still being formatted."""
    from ..pipeline.common import background
    check_strict_k(gamma.shape[1], strict)
    theta = doc_topics(gamma, strict)
    phi = word_topics(log_beta, strict)
    wnames = truncate_s20(word_names) if strict else list(word_names)
    n = native.lib()
    th_b = n.roundtrip_py2(np.ascontiguousarray(theta))
    ph_b = n.roundtrip_py2(np.ascontiguousarray(phi))
    dn = list(doc_names)

    def write():
        write_doc_results(doc_path, dn, theta)
        write_word_results(word_path, wnames, phi)
    return th_b, ph_b, wnames, background(write, "oni-lda-post-writer")


def _format_table(names, values, read_back):
    n = len(names)
    vals = np.ascontiguousarray(values, np.float64)
    back = np.empty_like(vals) if read_back else None
    text = native.lib().format_rows(None, [("dict", list(names), np.arange(n, dtype=np.int32)),
                                           ("py2row", vals, " ", back)], n=n)
    return text, back


def export_sharded(ctx, doc_names, gamma, word_names, log_beta, doc_path, word_path, strict=True,
                   read_back: bool = False, gather: bool = True, num_words: int = None):
    """``export`` with every rank writing its own rows of both files (the row-sharded lda_post stage).

    ``doc_names`` / ``gamma``: this rank's documents (its contiguous block of doc.dat, in rank order);
    ``word_names`` / ``log_beta``: the whole vocabulary, on every rank.  doc_results.csv takes the
    ranks' document blocks in rank order; word_results.csv is split by vocabulary slice
    [V r / N, V (r + 1) / N).  lda_post.py normalises each topic by Python's sequential sum over all V
    words (lda_post.py:88-96): here rank r continues the running sums of ranks < r
    (``shardio.chain``), so the totals -- and every byte of both files -- equal the one-process
    export.  ``gather``: return the whole θ / φ read-back tables on every rank (the scorers' broadcast
    model, flow_post_lda.scala:112-123; the resume path); otherwise this rank's rows and the names of
    its vocabulary slice.  ``word_names``: every word, or (``gather=False``) only the slice
    [V r / N, V (r + 1) / N) with ``num_words`` = V."""
    from ..parallel import shardio as SIO
    N, r = SIO.world(ctx), SIO.rank(ctx)
    check_strict_k(log_beta.shape[0], strict)
    theta = doc_topics(gamma, strict)
    text, th_b = _format_table(doc_names, theta, read_back)
    SIO.write_segments(ctx, doc_path, [text])
    V = log_beta.shape[1]
    v0, v1 = V * r // N, V * (r + 1) // N
    lb = np.ascontiguousarray(np.asarray(log_beta, np.float64)[:, v0:v1])
    if strict:
        lb = native.lib().roundtrip_fixed10(lb)
    raw = np.exp(lb)
    K = raw.shape[0]
    total = SIO.chain(ctx, lambda carry: np.cumsum(np.concatenate([carry[:, None], raw], 1), 1)[:, -1],
                      np.zeros(K, np.float64))
    phi = np.ascontiguousarray((raw / total[:, None]).T)
    wn = list(word_names[v0:v1]) if num_words is None else list(word_names)
    if len(wn) != v1 - v0:
        raise ValueError(f"word names: {len(wn)} for the vocabulary slice [{v0}, {v1})")
    wnames = truncate_s20(wn) if strict else wn
    text, ph_b = _format_table(wnames, phi, read_back)
    SIO.write_segments(ctx, word_path, [text])
    th, ph = (th_b, ph_b) if read_back else (theta, phi)
    if not gather:
        # this rank's rows only: its documents' θ, its vocabulary slice's φ and the slice's names as
        # written (pipeline/common.py ShardedTables fetches the rows a scorer needs from their ranks)
        return th, ph, wnames
    th = np.concatenate(SIO.allgather_array(ctx, np.ascontiguousarray(th)))
    ph = np.concatenate(SIO.allgather_array(ctx, np.ascontiguousarray(ph)))
    all_names = truncate_s20(word_names) if strict else list(word_names)
    return th, ph, all_names


def read_results(path: str):
    """doc_results.csv / word_results.csv -> (keys, values [n, K]) as the Scala scorers parse them
    (key = field 0, values = field 1 with quotes removed, split on ' ', toDouble;
    flow_post_lda.scala:107-123).  Later duplicate keys win (collectAsMap)."""
    keys, vals = [], []
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            parts = line.split(",")
            keys.append(parts[0])
            vals.append([float(x) for x in parts[1].replace('"', "").split(" ")])
    return keys, np.asarray(vals, np.float64)
