"""Planted-LDA synthetic corpora with heavy-tailed document lengths.

Used by tests and micro-benchmarks of the LDA core in isolation.  Documents
follow the shape of oni-ml corpora: most "IP documents" hold a
handful of distinct words, a few servers / NAT gateways hold thousands.
"""
from __future__ import annotations

import numpy as np

from ..corpus.csr import Corpus


def planted_corpus(num_docs=2000, num_terms=500, num_topics=8, mean_tokens=30, tail=1.2, max_tokens=200_000,
                   doc_alpha=0.2, topic_eta=0.05, seed=0) -> Corpus:
    rng = np.random.default_rng(seed)
    # heavy-tailed token counts: Pareto body scaled to the requested mean
    raw = rng.pareto(tail, size=num_docs) + 1.0
    ntok = np.maximum(1, np.minimum(max_tokens, np.round(raw / raw.mean() * mean_tokens))).astype(np.int64)
    zipf = 1.0 / np.arange(1, num_terms + 1) ** 0.9
    phi = rng.dirichlet(topic_eta + 20 * zipf / zipf.sum(), size=num_topics)       # [K, V]
    theta = rng.dirichlet(np.full(num_topics, doc_alpha), size=num_docs)           # [D, K]
    total = int(ntok.sum())
    doc_of = np.repeat(np.arange(num_docs), ntok)
    # topic per token
    cth = np.cumsum(theta, axis=1)
    u = rng.random(total)
    z = (u[:, None] > cth[doc_of]).sum(1)
    z = np.minimum(z, num_topics - 1)
    # word per token by inverse CDF per topic
    cph = np.cumsum(phi, axis=1)
    w = np.empty(total, np.int64)
    u2 = rng.random(total)
    for k in range(num_topics):
        m = z == k
        w[m] = np.minimum(np.searchsorted(cph[k], u2[m] * cph[k, -1]), num_terms - 1)
    key = doc_of.astype(np.int64) * num_terms + w
    uk, cnt = np.unique(key, return_counts=True)
    d = uk // num_terms
    ww = (uk % num_terms).astype(np.int32)
    ptr = np.zeros(num_docs + 1, np.int64)
    np.cumsum(np.bincount(d, minlength=num_docs), out=ptr[1:])
    # keep only used words (lda-c: num_terms = max id + 1); remap densely
    used = np.unique(ww)
    remap = np.full(num_terms, -1, np.int64)
    remap[used] = np.arange(used.size)
    return Corpus(ptr, remap[ww].astype(np.int32), cnt.astype(np.int64), int(used.size),
                  meta=dict(kind="planted", seed=seed))
