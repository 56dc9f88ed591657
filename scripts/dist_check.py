#!/usr/bin/env python
"""Multi-rank EM check (one process per rank, torchrun): the HIP engine with document sharding
and the class_word reduction (ONI_DIST_EXCHANGE = dense | sparse | auto).  Prints one JSON line
(rank 0) with the likelihood trajectory, alpha, a checksum of the full model and the exchange mode.

On one GPU several ranks rehearse the multi-GPU path over gloo (ONI_DIST_BACKEND=gloo; the
sparse all-to-all is staged through host memory there); with one GPU per rank it runs RCCL.
With WORLD_SIZE unset it runs single-process (the reference trajectory)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oni_ml_amd.corpus.csr import Corpus  # noqa: E402
from oni_ml_amd.models.lda.em import LDAEngine  # noqa: E402
from oni_ml_amd.models.lda.settings import LDASettings  # noqa: E402
from oni_ml_amd.parallel import dist as D  # noqa: E402
from oni_ml_amd.synth.corpus import planted_corpus  # noqa: E402


def shifted_vocab(c):
    """Second half of the documents on (mostly) disjoint word ids: shards share ~10% of words."""
    w = c.word_idx.copy()
    half = c.doc_ptr[c.num_docs // 2]
    tail = w[half:]
    w[half:] = np.where(tail % 10 == 0, tail, tail + c.num_terms)
    return Corpus(c.doc_ptr.copy(), w, c.counts.copy(), 2 * c.num_terms)


def main():
    K = int(os.environ.get("DIST_CHECK_K", "20"))
    ctx = D.init_from_env()
    c = shifted_vocab(planted_corpus(num_docs=3000, num_terms=2000, num_topics=8, mean_tokens=40, tail=1.0,
                                     max_tokens=20_000, seed=4))
    eng = LDAEngine(c, K, LDASettings(em_max_iter=6), backend="hip", dist=ctx if ctx.active else None,
                    seed=3, precision=os.environ.get("DIST_CHECK_PRECISION", "fp64"))
    res = eng.run()
    lb = eng.log_beta()
    g = eng.gather_gamma()
    if ctx.rank == 0:
        print(json.dumps(dict(world=ctx.world_size, exchange=eng.exchange_mode,
                              rows=None if eng._xchg is None else eng._xchg.rows,
                              likelihoods=[x[0] for x in res.likelihoods], alpha=eng.alpha,
                              beta_sum=float(np.exp(lb).sum()), beta_checksum=float((lb * np.arange(lb.shape[1])).sum()),
                              gamma_sum=float(g.sum()), gamma_shape=list(g.shape), precision=eng.precision)),
              flush=True)
    ctx.shutdown()


if __name__ == "__main__":
    main()
