"""lda-c / oni-ml on-disk formats.

Writers go through the multithreaded C++ formatter (`_oninative.write_rows`) so
100M-row outputs are not Python-bound; readers use numpy.

| file              | format                                              | reference            |
|-------------------|-----------------------------------------------------|----------------------|
| words.dat         | ``wid,word`` (0-based)                              | lda_pre.py:36-41     |
| doc.dat           | ``did,ip`` (1-based)                                | lda_pre.py:59-72     |
| model.dat         | ``N wid:cnt wid:cnt ...``                           | lda_pre.py:89-94     |
| <tag>.beta        | K lines x V values ``" %5.10f"``                    | lda-c save_lda_model |
| <tag>.gamma       | D lines, ``"%5.10f"`` joined by single spaces       | lda-c save_gamma     |
| <tag>.other       | ``num_topics K / num_terms V / alpha a``            | lda-c save_lda_model |
| likelihood.dat    | ``"%10.10f\\t%5.5e"`` per EM iteration              | lda-c run_em         |
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np

from ..corpus.csr import Corpus
from ..ops import native


def _n():
    return native.lib()


def write_words_dat(path: str, names: Sequence[str]):
    n = len(names)
    _n().write_rows(path, None, [("int", np.arange(n, dtype=np.int64)), ("dict", list(names), np.arange(n, dtype=np.int32))], n=n)


def write_doc_dat(path: str, names: Sequence[str]):
    n = len(names)
    _n().write_rows(path, None, [("int", np.arange(1, n + 1, dtype=np.int64)), ("dict", list(names), np.arange(n, dtype=np.int32))], n=n)


def read_index_file(path: str) -> List[str]:
    """words.dat / doc.dat -> names in file order (the index column is implied by position)."""
    out = []
    with open(path, "r", encoding="utf-8", newline="") as f:
        for line in f:
            line = line.rstrip("\n").rstrip("\r")
            if not line:
                continue
            i = line.find(",")
            out.append(line[i + 1:])
    return out


def write_model_dat(path: str, c: Corpus):
    """lda-c corpus format, one document per line (multithreaded C++ writer)."""
    _n().write_ldac_corpus(path, np.asarray(c.doc_ptr, np.int64), np.asarray(c.word_idx, np.int32),
                           np.asarray(c.counts, np.int64))


def read_model_dat(path: str) -> Corpus:
    """Parse lda-c corpus format; num_terms = max word id + 1 (lda-c read_data)."""
    ptr, w, cnt = _n().read_ldac_corpus(path)
    return Corpus(ptr, w, cnt, int(w.max()) + 1 if w.size else 0)


def save_beta(path: str, log_beta: np.ndarray):
    """K x V log p(w|z), each value as ' %5.10f'."""
    lb = np.ascontiguousarray(log_beta, dtype=np.float64)
    K = lb.shape[0]
    _n().write_rows(path, None, [("const", ""), ("fixedrow", lb, " ")], sep=" ", n=K)


def save_gamma(path: str, gamma: np.ndarray):
    g = np.ascontiguousarray(gamma, dtype=np.float64)
    _n().write_rows(path, None, [("fixedrow", g, " ")], n=g.shape[0])


def save_other(path: str, K: int, V: int, alpha: float):
    with open(path, "w") as f:
        f.write(f"num_topics {K} \nnum_terms {V} \nalpha {alpha:5.10f} \n")


def save_model(prefix: str, log_beta: np.ndarray, alpha: float):
    save_beta(prefix + ".beta", log_beta)
    save_other(prefix + ".other", log_beta.shape[0], log_beta.shape[1], alpha)


def load_other(path: str) -> dict:
    out = {}
    with open(path) as f:
        for line in f:
            p = line.split()
            if len(p) >= 2:
                out[p[0]] = float(p[1]) if p[0] == "alpha" else int(p[1])
    return out


def load_beta(path: str) -> np.ndarray:
    return np.atleast_2d(np.loadtxt(path, dtype=np.float64))


def load_gamma(path: str) -> np.ndarray:
    return np.atleast_2d(np.loadtxt(path, dtype=np.float64))


def load_model(prefix: str):
    """(log_beta [K, V], alpha) from <prefix>.beta / <prefix>.other (lda-c load_lda_model)."""
    o = load_other(prefix + ".other")
    lb = load_beta(prefix + ".beta")
    if lb.shape != (o["num_topics"], o["num_terms"]):
        raise ValueError(f"{prefix}.beta shape {lb.shape} != .other ({o['num_topics']}, {o['num_terms']})")
    return lb, float(o["alpha"])


def append_likelihood(path: str, likelihood: float, conv: float):
    with open(path, "a") as f:
        f.write(f"{likelihood:10.10f}\t{conv:5.5e}\n")


def format_likelihood_line(likelihood: float, conv: float) -> str:
    return f"{likelihood:10.10f}\t{conv:5.5e}\n"


def write_settings(path: str, settings):
    with open(path, "w") as f:
        f.write(settings.dumps())
