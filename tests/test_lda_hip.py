"""Numerics of the gfx950 kernels the fp64 engine shares: scoring, the alpha Newton and the device EM
loop control (against float64 host / PyTorch references)."""
import math

import numpy as np
import pytest
import torch

from oni_ml_amd.models.lda import special
from oni_ml_amd.models.lda.em import LDAEngine
from oni_ml_amd.models.lda.settings import LDASettings
from oni_ml_amd.ops import reference as R
from oni_ml_amd.synth.corpus import planted_corpus

pytestmark = pytest.mark.gpu


def test_device_convergence_matches_host_loop():
    """EM run with the lda-c loop test on the device (batches of 8 replays, stopping mid-batch)
    = the same run with one iteration per read-back: identical history, alpha and gamma."""
    c = planted_corpus(num_docs=2500, num_terms=700, num_topics=6, seed=13)
    res = []
    for batch in (1, 8):
        eng = LDAEngine(c, 20, LDASettings(em_max_iter=60, em_converged=2e-4), backend="hip", seed=9)
        eng.max_batch = eng.pipe_batch = batch   # (run() without saves batches by pipe_batch)
        r = eng.run()
        res.append((r.likelihoods, eng.alpha, eng.gather_gamma(), r.em_iterations))
    (L1, a1, g1, n1), (L8, a8, g8, n8) = res
    assert n1 == n8 and 3 <= n1 < 60
    assert L1 == L8 and a1 == a8
    assert np.array_equal(g1, g8)
    # host recomputation of the loop test over the recorded history
    Lold = 0.0
    for i, (lik, conv) in enumerate(L1, start=1):
        want = (Lold - lik) / Lold if Lold != 0 else math.inf
        assert conv == want
        Lold = lik
    assert not (L1[-1][1] > 2e-4 or L1[-1][1] < 0)


def test_score_kernel_bitwise(hip):
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(0)
    D, V, K, n = 50, 80, 20, 5000
    theta = torch.rand(D, K, generator=gen, dtype=torch.float64)
    theta /= theta.sum(1, keepdim=True)
    phi = torch.rand(V, K, generator=gen, dtype=torch.float64) * 1e-3
    da = torch.randint(-1, D, (n,), generator=gen, dtype=torch.int32)
    wa = torch.randint(-1, V, (n,), generator=gen, dtype=torch.int32)
    db = torch.randint(-1, D, (n,), generator=gen, dtype=torch.int32)
    wb = torch.randint(-1, V, (n,), generator=gen, dtype=torch.int32)
    out = hip.score_events(theta.to(dev), phi.to(dev), K, 0.05, da.to(dev), wa.to(dev), db.to(dev), wb.to(dev), 1e-4)
    ref = R.score(theta, phi, K, 0.05, da, wa, db, wb, 1e-4)
    for a, b in zip(out, ref):
        assert torch.equal(a.cpu(), b), "scores must match the sequential f64 reference bit for bit"


@pytest.mark.parametrize("K", [20, 50, 100])
def test_alpha_newton_device_matches_host(K):
    """Device lda-c opt_alpha (two lanes) == host special.opt_alpha, and the lgamma constant."""
    from oni_ml_amd.ops import hip as H
    D = 124451
    for astar in (0.03, 0.2, 1.0, 2.5, 7.0):
        ss = -D * (K * special.digamma(K * astar) - K * special.digamma(astar)) * 1.01
        scal = torch.tensor([0.0, ss], dtype=torch.float64, device="cuda")
        params = torch.zeros(H.PARAM_COUNT, dtype=torch.float64, device="cuda")
        params[0] = 2.5
        out = torch.zeros(1, dtype=torch.float64, device="cuda")
        H.alpha_newton(scal, D, K, True, params, out)
        torch.cuda.synchronize()
        host = special.opt_alpha(ss, D, K)
        a = float(out.item())
        assert a == pytest.approx(host, rel=1e-9), (astar, a, host)
        assert float(params[1].item()) == pytest.approx(special.lik_const(a, K), rel=1e-9, abs=1e-9)


@pytest.mark.parametrize("V,K,KS", [(1000, 20, 20), (777, 50, 52), (4097, 100, 100), (3, 7, 8)])
def test_log_beta_kernel_bitwise(hip, V, K, KS):
    """The saved log beta's HIP kernel (ops/hip.py log_beta_t) against torch's transpose / log / where chain on
    the device, bit for bit, including the -100 floor of zero counts and padding columns past K."""
    from oni_ml_amd.ops import hip as H
    g = torch.Generator().manual_seed(V + K)
    cw = torch.rand((V, KS), generator=g, dtype=torch.float64) * 50
    cw[torch.rand((V, KS), generator=g) < 0.2] = 0.0
    cw = cw.cuda()
    ct = cw.sum(0) + 1.0
    got = H.log_beta_t(cw, ct, K, -100.0)
    cT = cw[:, :K].T.contiguous()
    want = torch.where(cT > 0, torch.log(cT) - torch.log(ct[:K])[:, None], torch.full_like(cT, -100.0))
    assert got.shape == (K, V)
    assert torch.equal(got.view(torch.int64), want.view(torch.int64))
