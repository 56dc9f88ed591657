"""Numerics of the gfx950 LDA kernels against the float64 PyTorch reference.

Most tests here cover the fp32 Jacobi engine (``--precision fp32``, lda_estep*.hip), an opt-in fast
mode with a documented model bias against lda-c (profiles/r2_precision_parity.md): they are marked
``experimental`` and run only with ONI_EXPERIMENTAL=1.  The kernels the fp64 product path shares
(scoring, the alpha Newton, the device EM loop control) are tested unconditionally."""
import math

import numpy as np
import pytest
import torch

from oni_ml_amd.corpus.csr import Corpus, DeviceCorpus
from oni_ml_amd.models.lda import special
from oni_ml_amd.models.lda.em import LDAEngine, _Buckets
from oni_ml_amd.models.lda.settings import LDASettings
from oni_ml_amd.ops import reference as R
from oni_ml_amd.synth.corpus import planted_corpus

pytestmark = pytest.mark.gpu


def _corpus_with_long_docs(seed=3):
    # heavy tail so every bucket (G16 ... B8) is populated
    return planted_corpus(num_docs=1500, num_terms=3000, num_topics=6, mean_tokens=60, tail=0.9,
                          max_tokens=400_000, seed=seed)


def _random_beta(V, K, KS, seed=0, dev="cuda"):
    rng = np.random.default_rng(seed)
    cw = 1.0 / V + rng.random((V, K))
    b = cw / cw.sum(0, keepdims=True)
    out = torch.zeros(V, KS, dtype=torch.float32)
    out[:, :K] = torch.from_numpy(b).float()
    return out.to(dev)


@pytest.mark.parametrize("K,vconv,wide", [(20, -1e30, None), (7, -1e30, None), (50, -1e30, None), (100, -1e30, None),
                                          (20, 1e-6, None), (30, -1e30, "1"), (30, -1e30, "0"), (64, -1e30, None),
                                          (128, -1e30, None), (100, 1e-6, None), (50, -1e30, "0")])
@pytest.mark.experimental
def test_estep_matches_reference(hip, K, vconv, wide, monkeypatch):
    """Every length bucket of the narrow (K <= 32) and wide-topic (K > 32, lda_estep_wide.hip)
    E-step kernels against the fp64 Jacobi oracle; ``wide`` forces a layout (ONI_ESTEP_WIDE)."""
    if wide is not None:
        monkeypatch.setenv("ONI_ESTEP_WIDE", wide)
    c = _corpus_with_long_docs()
    dev = torch.device("cuda")
    KS = hip.padded_topics(K)
    dc = DeviceCorpus.build(c, dev)
    beta = _random_beta(c.num_terms, K, KS, seed=K)
    D, nnz = c.num_docs, c.nnz
    gamma = torch.zeros(D, KS, device=dev)
    e = torch.zeros(D, KS, device=dev)
    r = torch.zeros(nnz, device=dev)
    lik = torch.zeros(D, dtype=torch.float64, device=dev)
    ass = torch.zeros(D, dtype=torch.float64, device=dev)
    iters = torch.zeros(D, dtype=torch.int32, device=dev)
    # vconv = -1e30 runs exactly vmax Jacobi iterations per doc (tight fp32-vs-fp64
    # numerics); vconv = 1e-6 is the lda-c convergence rule, where a doc may stop one
    # iteration apart in fp32 and fp64, so gamma is compared loosely there.
    alpha, vmax = 0.7, 20
    lc = special.lik_const(alpha, K)
    plan = _Buckets(dc.doc_len, KS, dev, "doc").plan
    assert len(plan) >= 4
    for var, order in plan:
        hip.lda_estep(dc.doc_ptr, dc.word_idx, dc.counts, order, beta, K, alpha, lc, vmax, vconv, gamma, e, r,
                      lik, ass, iters, var)
    torch.cuda.synchronize()
    ref = R.estep_jacobi(dc.doc_ptr, dc.word_idx, dc.counts, beta.double(), K, alpha, vmax, vconv)
    g, gr = gamma[:, :K].double(), ref["gamma"]
    rel = ((g - gr).abs() / gr.abs().clamp_min(1e-3)).max().item()
    assert rel < (2e-3 if vconv < 0 else 2e-2), rel
    lrel = ((lik - ref["lik"]).abs() / ref["lik"].abs()).max().item()
    assert lrel < 1e-4, lrel
    assert abs(lik.sum().item() - ref["lik"].sum().item()) / abs(ref["lik"].sum().item()) < 1e-5
    # padding topics stay zero
    if KS > K:
        assert gamma[:, K:].abs().max().item() == 0
    # iteration counts agree for the vast majority of documents
    agree = (iters.cpu() == ref["iters"].cpu()).float().mean().item()
    # with the lda-c rule a doc stops when the relative change is <= 1e-6, which is at the
    # fp32 resolution of its likelihood: fp32 and fp64 may stop one iteration apart
    assert agree > (0.999 if vconv < 0 else 0.75), agree
    # alpha sufficient statistic
    arel = ((ass - ref["alpha_ss"]).abs() / ref["alpha_ss"].abs().clamp_min(1.0)).max().item()
    assert arel < 1e-3, arel
    if vconv < 0:
        # E of the final phi and r_n = c_n / P_n under it (the suff-stats inputs)
        erel = ((e[:, :K].double() - ref["e"]).abs() / ref["e"].abs().clamp_min(1e-6)).max().item()
        assert erel < 2e-3, erel
        rrel = ((r.double() - ref["r"]).abs() / ref["r"].abs().clamp_min(1e-30)).max().item()
        assert rrel < 2e-3, rrel


@pytest.mark.experimental
def test_suffstats_and_mstep(hip):
    c = _corpus_with_long_docs(seed=5)
    K = 20
    dev = torch.device("cuda")
    KS = hip.padded_topics(K)
    dc = DeviceCorpus.build(c, dev)
    beta = _random_beta(c.num_terms, K, KS, seed=1)
    D, nnz, V = c.num_docs, c.nnz, c.num_terms
    gen = torch.Generator(device="cpu").manual_seed(0)
    e = torch.rand(D, KS, generator=gen).to(dev)
    e[:, K:] = 0
    r = torch.rand(nnz, generator=gen).to(dev)
    cw = torch.zeros(V, KS, device=dev)
    for var, order in _Buckets(dc.word_len, KS, dev, "word").plan:
        hip.lda_suffstats(dc.word_ptr, dc.csc_ent, dc.csc_doc, order, e, r, beta, cw, var)
    ref = R.suffstats(dc.doc_ptr, dc.word_idx, e.double(), r.double(), beta.double(), V, K)
    rel = ((cw[:, :K].double() - ref).abs() / ref.abs().clamp_min(1e-20)).max().item()
    assert rel < 1e-4, rel
    # determinism: bitwise identical on a second run
    cw2 = torch.zeros_like(cw)
    for var, order in _Buckets(dc.word_len, KS, dev, "word").plan:
        hip.lda_suffstats(dc.word_ptr, dc.csc_ent, dc.csc_doc, order, e, r, beta, cw2, var)
    assert torch.equal(cw, cw2)
    # M-step
    cw[5, 3] = 0.0
    ct = cw.sum(0, dtype=torch.float64)
    b2 = torch.empty_like(cw)
    hip.lda_mstep(cw, ct, b2, K)
    refb = R.mstep(cw.double(), ct, K)
    assert torch.allclose(b2[:, :K].double(), refb, rtol=1e-6, atol=1e-45)
    # lda-c's floor log p = -100 becomes the f32 subnormal nearest exp(-100): 27 * 2^-149 = 3.7835e-44,
    # 1.7 % above exp(-100) = 3.7201e-44 (the fp64 engine keeps exp(-100) exactly)
    assert b2[5, 3].item() == torch.tensor(math.exp(-100), dtype=torch.float32).item() == 27 * 2.0 ** -149
    if KS > K:
        assert b2[:, K:].abs().max().item() == 0


@pytest.mark.experimental
@pytest.mark.parametrize("K,wide", [(20, False), (30, True), (50, True), (100, True), (128, True)])
def test_suffstats_fused_and_partial_colsums(hip, K, wide):
    """Single-launch suff-stats (heavy / medium / light words, empty words included) against the
    fp64 reference, bitwise reproducible; the per-workgroup column sums give the class totals.
    wide: the wide-topic layout (lda_suff_wide, 4 or 8 lanes per CSC entry) used for K > 32."""
    # Zipf-like word usage: a few "stop words" in most documents (heavy), a middle band, a long
    # tail of rare words and some never-used ones (empty)
    rng = np.random.default_rng(6)
    D, V = 3000, 4000
    p = 1.0 / np.arange(1, V + 1) ** 1.1
    p[-200:] = 0
    p /= p.sum()
    ptr, idx = [0], []
    for _ in range(D):
        n = int(rng.integers(1, 60))
        w = np.unique(rng.choice(V, size=n, p=p))
        idx.append(w)
        ptr.append(ptr[-1] + w.size)
    idx = np.concatenate(idx)
    c = Corpus(np.array(ptr), idx, rng.integers(1, 5, idx.size), V)
    dev = torch.device("cuda")
    KS = hip.padded_topics(K)
    dc = DeviceCorpus.build(c, dev)
    beta = _random_beta(c.num_terms, K, KS, seed=2)
    D, nnz, V = c.num_docs, c.nnz, c.num_terms
    gen = torch.Generator(device="cpu").manual_seed(1)
    e = torch.rand(D, KS, generator=gen).to(dev)
    e[:, K:] = 0
    r = torch.rand(nnz, generator=gen).to(dev)
    plan = hip.SuffPlan(dc.word_len, dev, wide=wide)
    assert plan.n_heavy > 0 and plan.n_medium > 0 and plan.n_light > 0 and int((dc.word_len == 0).sum()) > 0
    part = torch.zeros(plan.n_blocks, KS, dtype=torch.float64, device=dev)
    cw = torch.full((V, KS), float("nan"), device=dev)          # every row must be written
    hip.lda_suffstats_fused(dc.word_ptr, dc.csc_ent, dc.csc_doc, plan, e, r, beta, cw, part)
    ref = R.suffstats(dc.doc_ptr, dc.word_idx, e.double(), r.double(), beta.double(), V, K)
    assert not torch.isnan(cw).any()
    rel = ((cw[:, :K].double() - ref).abs() / ref.abs().clamp_min(1e-20)).max().item()
    assert rel < 1e-4, rel
    ct = torch.zeros(KS, dtype=torch.float64, device=dev)
    hip.colsum_partials(part, plan.n_blocks, ct)
    assert torch.allclose(ct, cw.double().sum(0), rtol=1e-12)
    cw2 = torch.zeros_like(cw)
    part2 = torch.zeros_like(part)
    hip.lda_suffstats_fused(dc.word_ptr, dc.csc_ent, dc.csc_doc, plan, e, r, beta, cw2, part2)
    assert torch.equal(cw, cw2) and torch.equal(part, part2)
    # [lik, alpha_ss | topics] partial layout: the document-slice sums ride in columns 0 / 1
    lik = torch.rand(D, generator=gen, dtype=torch.float64).to(dev) - 0.5
    ass = torch.rand(D, generator=gen, dtype=torch.float64).to(dev) * -3.0
    part3 = torch.full((plan.n_blocks, KS + 2), float("nan"), dtype=torch.float64, device=dev)
    cw4 = torch.zeros_like(cw)
    hip.lda_suffstats_fused(dc.word_ptr, dc.csc_ent, dc.csc_doc, plan, e, r, beta, cw4, part3, scalars=(lik, ass, 0, D))
    assert torch.equal(cw4, cw) and torch.equal(part3[:, 2:], part)
    red = torch.zeros(KS + 2, dtype=torch.float64, device=dev)
    hip.colsum_partials(part3, plan.n_blocks, red)
    assert torch.equal(red[2:], ct)
    assert red[0].item() == pytest.approx(lik.sum().item(), rel=1e-12)
    assert red[1].item() == pytest.approx(ass.sum().item(), rel=1e-12)
    hip.lda_suffstats_fused(dc.word_ptr, dc.csc_ent, dc.csc_doc, plan, e, r, beta, cw4, part3)   # no slice: zeros
    assert part3[:, :2].abs().max().item() == 0
    # a set gate skips the launch
    gate = torch.ones(1, dtype=torch.float64, device=dev)
    cw3 = torch.zeros_like(cw)
    hip.lda_suffstats_fused(dc.word_ptr, dc.csc_ent, dc.csc_doc, plan, e, r, beta, cw3, part2, gate=gate)
    assert cw3.abs().max().item() == 0


def test_device_convergence_matches_host_loop():
    """EM run with the lda-c loop test on the device (batches of 8 replays, stopping mid-batch)
    = the same run with one iteration per read-back: identical history, alpha and gamma."""
    c = planted_corpus(num_docs=2500, num_terms=700, num_topics=6, seed=13)
    res = []
    for batch in (1, 8):
        eng = LDAEngine(c, 20, LDASettings(em_max_iter=60, em_converged=2e-4), backend="hip", seed=9)
        eng.max_batch = batch
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


@pytest.mark.experimental
def test_em_hip_tracks_torch_reference():
    c = planted_corpus(num_docs=2000, num_terms=600, num_topics=8, seed=11)
    st = LDASettings(em_max_iter=8)
    hip_eng = LDAEngine(c, 20, st, backend="hip", seed=4, precision="fp32")
    ref_eng = LDAEngine(c, 20, LDASettings(em_max_iter=8), backend="torch", device="cuda", seed=4)
    r1 = hip_eng.run()
    r2 = ref_eng.run()
    L1 = np.array([x[0] for x in r1.likelihoods])
    L2 = np.array([x[0] for x in r2.likelihoods])
    assert L1.shape == L2.shape
    assert np.max(np.abs(L1 - L2) / np.abs(L2)) < 1e-3
    assert abs(hip_eng.alpha - ref_eng.alpha) / ref_eng.alpha < 1e-2
    # likelihood increases (EM monotone up to var-inference slack)
    assert L1[-1] > L1[0]


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


@pytest.mark.experimental
@pytest.mark.parametrize("K", [20, 50, 100])
def test_split_documents_match_single_workgroup(hip, K):  # K = 50, 100: wide-topic split kernel
    """Huge documents split across workgroups (per-iteration cross-workgroup reduction) give the
    same E-step as the one-workgroup kernel and the fp64 reference."""
    c = planted_corpus(num_docs=400, num_terms=20000, num_topics=6, mean_tokens=400, tail=0.7,
                       max_tokens=2_000_000, seed=8)
    assert c.lengths().max() > 4 * 1024
    st = LDASettings(var_max_iter=15, var_converged=-1e30)
    outs = []
    for split in (True, False):
        eng = LDAEngine(c, K, st, backend="hip", seed=1, split_docs=split, precision="fp32")
        eng.init_random()
        if split:
            assert eng.doc_buckets.split is not None and eng.doc_buckets.split.batches
        sc = eng.e_step()
        torch.cuda.synchronize()
        if split:
            assert int(eng.doc_buckets.split.batches[0]["error"].item()) == 0
        outs.append((eng.gamma[:, :K].double().cpu(), eng.lik.cpu(), sc.cpu(), eng.cw.cpu(), eng.iters.cpu()))
    (g1, l1, s1, cw1, i1), (g0, l0, s0, cw0, i0) = outs
    assert torch.equal(i1, i0)
    rel = ((g1 - g0).abs() / g0.abs().clamp_min(1e-3)).max().item()
    assert rel < 2e-3, rel
    assert ((l1 - l0).abs() / l0.abs()).max().item() < 1e-5
    assert ((cw1 - cw0).abs().max() / cw0.abs().max()).item() < 1e-3
    ref = R.estep_jacobi(torch.from_numpy(c.doc_ptr), torch.from_numpy(c.word_idx), torch.from_numpy(c.counts).double(),
                         eng.beta.double().cpu(), K, eng.alpha, 15, -1e30)
    assert ((g1 - ref["gamma"]).abs() / ref["gamma"].abs().clamp_min(1e-3)).max().item() < 2e-3


@pytest.mark.experimental
@pytest.mark.parametrize("K", [3, 13, 24, 33, 77, 128])
def test_estep_random_corpora_edge_cases(hip, K):
    """Randomised corpora with the shapes real featurization produces: empty documents, duplicate
    (doc, word) entries (strict mode keeps the src/dst halves apart), counts > 1, words never used,
    every length bucket (and split documents); odd K (padding topics).  Every E-step kernel and
    the suff-stats against the fp64 references, fixed variational iterations."""
    rng = np.random.default_rng(K)
    V, D = 1500, 900
    lens = np.minimum(rng.zipf(1.4, D), 9000)
    lens[rng.choice(D, 25, replace=False)] = 0                      # empty documents
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = rng.integers(0, V - 100, int(ptr[-1]))                  # the last 100 words never occur
    for d in rng.choice(np.flatnonzero(lens > 3), 40, replace=False):  # duplicated entries
        a = ptr[d]
        words[a + 1] = words[a]
    counts = rng.integers(1, 4, words.size)
    c = Corpus(ptr.astype(np.int64), words.astype(np.int32), counts.astype(np.int64), V)
    dev = torch.device("cuda")
    eng = LDAEngine(c, K, LDASettings(var_max_iter=8, var_converged=-1e30), backend="hip", seed=K, split_min=2048,
                    precision="fp32")
    eng.init_random()
    eng.e_step()
    torch.cuda.synchronize()
    dc = eng.dc
    ref = R.estep_jacobi(dc.doc_ptr, dc.word_idx, dc.counts, eng.beta.double(), K, eng.alpha, 8, -1e30)
    g, gr = eng.gamma[:, :K].double(), ref["gamma"]
    assert ((g - gr).abs() / gr.abs().clamp_min(1e-3)).max().item() < 2e-3
    lik = eng.lik
    # per-document likelihoods near 0 (empty documents: lnG(Ka) - K lnG(a) - lnG(Ka) + K lnG(a)) carry the
    # fp32 rounding of the K-term topic phase, ~1e-4 absolute at K = 77: compare them absolutely
    assert ((lik - ref["lik"]).abs() / ref["lik"].abs().clamp_min(10.0)).max().item() < 1e-4
    nz = lens > 0
    rr = (eng.r.double() - ref["r"]).abs() / ref["r"].abs().clamp_min(1e-30)
    assert rr.max().item() < 2e-3
    if eng.KS > K:
        assert eng.gamma[:, K:].abs().max().item() == 0
    # suff-stats of that E-step (local statistics) against the fp64 scatter
    cw_ref = R.suffstats(dc.doc_ptr, dc.word_idx, eng.e[:, :K].double(), eng.r.double(), eng.beta.double(), V, K)
    cw = eng._cw_local[:, :K].double()
    rel = ((cw - cw_ref).abs() / cw_ref.abs().clamp_min(1e-20)).max().item()
    assert rel < 1e-4, rel
    assert cw[V - 100:].abs().max().item() == 0                      # unused words: zero rows
    assert int(nz.sum()) < D


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


@pytest.mark.experimental
def test_split_launch_cap_from_occupancy(hip, monkeypatch):
    """Split launches are sized from the occupancy API (co-residency of every segment of a launch);
    a forced small cap (ONI_SPLIT_MAX_BLOCKS) re-batches the huge documents and gives the same E-step."""
    cap = hip.split_launch_cap(20, False)
    assert 0 < cap <= hip.lib().split_max_blocks()
    assert hip.lib().split_capacity(20, False) >= cap and hip.lib().split_capacity(100, True) > 0
    c = planted_corpus(num_docs=300, num_terms=20000, num_topics=6, mean_tokens=400, tail=0.7,
                       max_tokens=2_000_000, seed=8)
    st = LDASettings(var_max_iter=10, var_converged=-1e30)
    outs = []
    for env in (None, "6"):
        if env:
            monkeypatch.setenv("ONI_SPLIT_MAX_BLOCKS", env)
        eng = LDAEngine(c, 20, st, backend="hip", seed=1, precision="fp32")
        sp = eng.doc_buckets.split
        if env:
            assert sp.max_blocks == 6 and all(b["n_blocks"] <= 6 for b in sp.batches)
        eng.init_random()
        eng.e_step()
        torch.cuda.synchronize()
        outs.append(eng.gamma[:, :20].double().cpu())
    assert torch.allclose(outs[0], outs[1], rtol=2e-3, atol=1e-4)
