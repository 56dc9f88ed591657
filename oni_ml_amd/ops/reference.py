"""Pure-PyTorch reference implementations of the LDA hot ops.

The `torch` LDA backend: a vectorised Jacobi fixed-point E-step (every word's phi from one digamma
vector per variational iteration; the closed-form likelihood and lda-c's convergence rule) across
documents with per-document convergence masks, plus the suff-stats and M-step.  It is a test rehearsal
engine only -- the one whose multi-rank statistics can fold bitwise like one process
(ONI_DIST_DETERMINISTIC=chain, tests/test_sharded_pipeline.py).  The MI355X engine is the fp64 block
Gauss-Seidel of csrc/hip/lda_gs64.hip and the CPU engine the lda-c Gauss-Seidel of
csrc/native/lda_ref.cpp; both are checked against lda_ref.cpp, not against this module.
"""
from __future__ import annotations

import math

import torch

from ..models.lda.special import digamma


def estep_jacobi(doc_ptr, word_idx, counts, beta, K, alpha, var_max_iter, var_conv, dtype=torch.float64,
                 chunk_docs=None):
    """Vectorised Jacobi variational E-step.

    Args:
      doc_ptr [D+1] int, word_idx [nnz] int, counts [nnz] float, beta [V, >=K]
      (exp log p(w|z), word-major).
    Returns dict(gamma [D,K], e [D,K], r [nnz], lik [D] f64, alpha_ss [D] f64, iters [D] int32).
    """
    dev = beta.device
    D = doc_ptr.numel() - 1
    nnz = word_idx.numel()
    doc_ptr = doc_ptr.to(dev, torch.int64)
    lens = doc_ptr[1:] - doc_ptr[:-1]
    doc_of = torch.repeat_interleave(torch.arange(D, device=dev), lens)
    widx = word_idx.to(dev, torch.int64)
    c = counts.to(dev, dtype)
    B = beta[:, :K].to(dtype)[widx]                       # [nnz, K]
    total = torch.zeros(D, dtype=torch.float64, device=dev).index_add_(0, doc_of, counts.to(dev, torch.float64))
    a = torch.tensor(float(alpha), dtype=dtype, device=dev)
    lc = math.lgamma(K * alpha) - K * math.lgamma(alpha)

    gam = (a + (total / K).to(dtype)).unsqueeze(1).expand(D, K).clone()
    psi = digamma(gam)
    e_last = torch.zeros(D, K, dtype=dtype, device=dev)
    r_last = torch.zeros(nnz, dtype=dtype, device=dev)
    lik = torch.zeros(D, dtype=torch.float64, device=dev)
    lik_old = torch.zeros(D, dtype=torch.float64, device=dev)
    conv = torch.ones(D, dtype=torch.float64, device=dev)
    iters = torch.zeros(D, dtype=torch.int32, device=dev)
    dsum_last = digamma(gam.sum(1)).to(torch.float64)
    active = torch.ones(D, dtype=torch.bool, device=dev)
    it = 0
    while True:
        cont = active & (conv > float(var_conv))
        if var_max_iter >= 0:
            cont &= iters < var_max_iter
        if not bool(cont.any()):
            break
        active = cont
        it += 1
        m = psi.max(1, keepdim=True).values
        E = torch.exp(psi - m)                               # [D,K]
        P = (E[doc_of] * B).sum(1).clamp_min(1e-30)          # [nnz]
        r = c / P
        acc = torch.zeros(D, K, dtype=dtype, device=dev).index_add_(0, doc_of, r.unsqueeze(1) * B)
        lsum = torch.zeros(D, dtype=torch.float64, device=dev).index_add_(0, doc_of, (c * torch.log(P)).double())
        gn = a + E * acc
        S = gn.sum(1)
        dS = digamma(S)
        pn = digamma(gn)
        y = pn - dS.unsqueeze(1)
        term = ((a - 1) * y + torch.lgamma(gn) - (gn - 1) * y + (gn - a) * (pn - psi)).double().sum(1)
        L = lc - torch.lgamma(S).double() + term + (lsum + m.squeeze(1).double() * total) - total * dS.double()
        cv = (lik_old - L) / lik_old
        act = active
        act2 = act.unsqueeze(1)
        gam = torch.where(act2, gn, gam)
        psi = torch.where(act2, pn, psi)
        e_last = torch.where(act2, E, e_last)
        r_last = torch.where(act[doc_of], r, r_last)
        lik = torch.where(act, L, lik)
        conv = torch.where(act, cv, conv)
        lik_old = torch.where(act, L, lik_old)
        dsum_last = torch.where(act, dS.double(), dsum_last)
        iters = iters + act.to(torch.int32)
    ass = psi.double().sum(1) - K * dsum_last
    return dict(gamma=gam, e=e_last, r=r_last, lik=lik, alpha_ss=ass, iters=iters)


def suffstats(doc_ptr, word_idx, e, r, beta, V, K):
    """class_word [V, K] = beta * scatter(E[doc] * r) (deterministic order not guaranteed)."""
    dev = e.device
    D = doc_ptr.numel() - 1
    lens = (doc_ptr[1:] - doc_ptr[:-1]).to(dev, torch.int64)
    doc_of = torch.repeat_interleave(torch.arange(D, device=dev), lens)
    contrib = e[doc_of][:, :K] * r.unsqueeze(1)
    s = torch.zeros(V, K, dtype=e.dtype, device=dev).index_add_(0, word_idx.to(dev, torch.int64), contrib)
    return beta[:, :K].to(e.dtype) * s


def mstep(cw, class_total, K):
    """beta = cw/ct where cw > 0 else exp(-100)."""
    ct = class_total[:K].to(cw.dtype)
    out = torch.where(cw[:, :K] > 0, cw[:, :K] / ct, torch.full_like(cw[:, :K], math.exp(-100.0)))
    return out


def score(theta, phi, K, dflt, doc_a, word_a, doc_b=None, word_b=None, tol=float("inf")):
    """Reference scorer: sequential (non-fused) multiply-add over topics, float64."""
    def one(d, w):
        n = d.numel()
        s = torch.zeros(n, dtype=torch.float64, device=d.device)
        th = torch.where((d >= 0).unsqueeze(1), theta[d.clamp_min(0), :K], torch.full((n, K), dflt, dtype=torch.float64, device=d.device))
        ph = torch.where((w >= 0).unsqueeze(1), phi[w.clamp_min(0), :K], torch.full((n, K), dflt, dtype=torch.float64, device=d.device))
        for k in range(K):
            s = s + th[:, k] * ph[:, k]
        return s

    sa = one(doc_a.long(), word_a.long())
    sb = one(doc_b.long(), word_b.long()) if doc_b is not None else None
    key = torch.minimum(sa, sb) if sb is not None else sa
    return sa, sb, key, (key < tol).to(torch.uint8)


def flow_words(hour, minute, second, port_a, port_b, ipkt, ibyt, time_cuts, ibyt_cuts, ipkt_cuts):
    """Torch transcription of csrc/hip/flow_words.hip (flow_pre_lda.scala:272-358)."""
    t = (hour + minute / 60) + second / 3600
    def nb(v, c):
        return (v.unsqueeze(-1) > c.to(v.device).unsqueeze(0)).sum(-1).to(torch.int8)
    dp, sp = port_a, port_b                    # reference names: dport = col 10, sport = col 11
    mn, mx = torch.minimum(dp, sp), torch.maximum(dp, sp)
    c2 = ((dp <= 1024) | (sp <= 1024)) & ((dp > 1024) | (sp > 1024)) & (mn != 0)
    c3 = ~c2 & (dp > 1024) & (sp > 1024)
    c4a = ~c2 & ~c3 & (dp == 0) & (sp != 0)
    c4b = ~c2 & ~c3 & ~c4a & (sp == 0) & (dp != 0)
    c1 = ~(c2 | c3 | c4a | c4b)
    wp = torch.where(c2, mn, torch.where(c3, torch.full_like(mn, 333333.0), torch.where(
        c4a, sp, torch.where(c4b, dp, torch.where(mn == 0, mx, torch.full_like(mn, 111111.0))))))
    pc = torch.where(c2, 2, torch.where(c3, 3, torch.where(c4a | c4b, 4, 1))).to(torch.int8)
    # the reference's if / else-if chain for the "-1_" side
    r1 = c2 & (dp < sp)
    r2 = ~r1 & c2 & (sp < dp)
    r3 = ~r1 & ~r2 & (pc == 4) & (dp == 0)
    r4 = ~r1 & ~r2 & ~r3 & (pc == 4) & (sp == 0)
    dpre = r1 | r4
    spre = r2 | r3
    return dict(time=t, time_bin=nb(t, time_cuts), ibyt_bin=nb(ibyt, ibyt_cuts), ipkt_bin=nb(ipkt, ipkt_cuts),
                word_port=wp, p_case=pc, src_prefix=spre.to(torch.int8), dst_prefix=dpre.to(torch.int8))
