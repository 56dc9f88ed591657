"""lda-c special functions (utils.c) in float64 numpy/torch + the alpha Newton step.

Reference: oni-lda-c utils.c digamma/trigamma/log_sum and lda-alpha.c opt_alpha
(source absent from the mount, reconstructed from upstream
lda-c).  The same digamma series is used on the device (csrc/hip/common.h) so
host and device agree on the approximation, not just the function.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .settings import MAX_ALPHA_ITER, NEWTON_THRESH


def digamma(x):
    """lda-c digamma: shift by 6, asymptotic series, recurrence corrections."""
    if isinstance(x, torch.Tensor):
        x = x + 6.0
        p = 1.0 / (x * x)
        p = (((0.004166666666667 * p - 0.003968253986254) * p + 0.008333333333333) * p - 0.083333333333333) * p
        return (p + torch.log(x) - 0.5 / x - 1.0 / (x - 1) - 1.0 / (x - 2) - 1.0 / (x - 3)
                - 1.0 / (x - 4) - 1.0 / (x - 5) - 1.0 / (x - 6))
    x = np.asarray(x, dtype=np.float64) + 6.0
    p = 1.0 / (x * x)
    p = (((0.004166666666667 * p - 0.003968253986254) * p + 0.008333333333333) * p - 0.083333333333333) * p
    r = (p + np.log(x) - 0.5 / x - 1.0 / (x - 1) - 1.0 / (x - 2) - 1.0 / (x - 3)
         - 1.0 / (x - 4) - 1.0 / (x - 5) - 1.0 / (x - 6))
    return float(r) if r.ndim == 0 else r


def trigamma(x):
    x = float(x) + 6.0
    p = 1.0 / (x * x)
    p = (((((0.075757575757576 * p - 0.033333333333333) * p + 0.0238095238095238) * p
           - 0.033333333333333) * p + 0.166666666666667) * p + 1) / x + 0.5 * p
    for _ in range(6):
        x = x - 1
        p = 1.0 / (x * x) + p
    return p


def log_sum(log_a, log_b):
    if log_a < log_b:
        return log_b + math.log(1 + math.exp(log_a - log_b))
    return log_a + math.log(1 + math.exp(log_b - log_a))


def alhood(a, ss, D, K):
    return D * (math.lgamma(K * a) - K * math.lgamma(a)) + (a - 1) * ss


def d_alhood(a, ss, D, K):
    return D * (K * digamma(K * a) - K * digamma(a)) + ss


def d2_alhood(a, D, K):
    return D * (K * K * trigamma(K * a) - K * trigamma(a))


def opt_alpha(ss: float, D: int, K: int, init_a: float = 100.0) -> float:
    """Newton's method in log(alpha) (lda-alpha.c opt_alpha)."""
    log_a = math.log(init_a)
    it = 0
    while True:
        it += 1
        a = math.exp(log_a) if log_a < 709.78 else (math.nan if math.isnan(log_a) else math.inf)
        if math.isnan(a):
            init_a = init_a * 10
            a = init_a
            log_a = math.log(a)
        df = d_alhood(a, ss, D, K)
        d2f = d2_alhood(a, D, K)
        log_a = log_a - df / (d2f * a + df)
        if not (abs(df) > NEWTON_THRESH and it < MAX_ALPHA_ITER):
            break
    return math.exp(log_a) if log_a < 709.78 else (math.nan if math.isnan(log_a) else math.inf)


def lik_const(alpha: float, K: int) -> float:
    """lgamma(K*alpha) - K*lgamma(alpha), the doc-independent likelihood term."""
    return math.lgamma(alpha * K) - K * math.lgamma(alpha)
