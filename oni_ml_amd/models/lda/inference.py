"""`lda inf`: variational inference of held-out documents under a fixed model (lda-c infer).

Outputs <name>-gamma.dat (lda-c save_gamma format) and <name>-lda-lhood.dat
(one "%5.5f" document likelihood per line).
"""
from __future__ import annotations

import numpy as np
import torch

from ...io import ldac
from .em import LDAEngine, resolved_gs_updates
from .settings import LDASettings


def infer(corpus, log_beta: np.ndarray, alpha: float, settings: LDASettings, backend: str = "auto", device=None):
    """Returns (gamma [D, K] f64, per-document likelihood [D] f64).  The GPU engine runs the fp64 block
    Gauss-Seidel schedule; the cpu backend is lda-c's schedule (settings.gs_updates)."""
    K, V = log_beta.shape
    if corpus.num_terms > V:
        raise ValueError("corpus word id beyond the model vocabulary")
    corpus.num_terms = V
    eng = LDAEngine(corpus, K, settings, alpha_init=alpha, backend=backend, device=device)
    eng.init_from_model(log_beta, alpha)
    if eng.backend == "cpu":
        lb = np.ascontiguousarray(log_beta)
        r = eng._native.lda_estep_ldac(corpus.doc_ptr, corpus.word_idx, corpus.counts, lb, alpha,
                                       settings.var_max_iter, settings.var_converged, 1, 0,
                                       gs_updates=resolved_gs_updates(settings, K))
        lik = np.asarray(r["doc_likelihood"])
        return r["gamma"], lik
    eng.e_step()
    lik = eng.lik.double().cpu().numpy()
    return eng.local_gamma(), lik


def infer_files(settings_path: str, model_prefix: str, corpus_path: str, name: str, backend: str = "auto"):
    st = LDASettings.load(settings_path)
    lb, alpha = ldac.load_model(model_prefix)
    c = ldac.read_model_dat(corpus_path)
    g, lik = infer(c, lb, alpha, st, backend=backend)
    ldac.save_gamma(f"{name}-gamma.dat", g)
    with open(f"{name}-lda-lhood.dat", "w") as f:
        f.write("".join("%5.5f\n" % x for x in lik))
    return g, lik
