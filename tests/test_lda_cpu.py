"""LDA core on the CPU: lda-c reference numerics, Jacobi torch engine, lda CLI, resume."""
import math
import os
import subprocess
import sys

import numpy as np
import pytest
import scipy.special as sp
import torch

from oni_ml_amd.corpus.csr import Corpus
from oni_ml_amd.io import ldac
from oni_ml_amd.models.lda import special
from oni_ml_amd.models.lda.em import LDAEngine
from oni_ml_amd.models.lda.estimate import estimate
from oni_ml_amd.models.lda.settings import LDASettings
from oni_ml_amd.ops import native
from oni_ml_amd.ops import reference as R
from oni_ml_amd.synth.corpus import planted_corpus

N = native.lib()


def test_special_functions():
    for x in (0.05, 0.3, 1.0, 2.5, 17.0, 1234.5):
        assert N.digamma(x) == pytest.approx(sp.digamma(x), rel=1e-9, abs=1e-9)
        assert special.digamma(x) == pytest.approx(N.digamma(x), rel=1e-15)
        assert N.trigamma(x) == pytest.approx(sp.polygamma(1, x), rel=1e-8)
        assert special.trigamma(x) == pytest.approx(N.trigamma(x), rel=1e-14)
    assert N.log_sum(-3.0, -2.0) == pytest.approx(math.log(math.exp(-3) + math.exp(-2)))


@pytest.mark.parametrize("D,K,ss", [(100, 20, -8000.0), (5000, 10, -150000.0), (50, 5, -600.0)])
def test_opt_alpha_is_newton_root(D, K, ss):
    a = N.opt_alpha(ss, D, K)
    assert special.opt_alpha(ss, D, K) == pytest.approx(a, rel=1e-12)
    # stationary point of alhood(a) = D(lnG(Ka) - K lnG(a)) + (a-1) ss
    d = D * (K * sp.digamma(K * a) - K * sp.digamma(a)) + ss
    assert abs(d) < 1e-4 * D


def _ldac_inference_py(words, counts, lb, alpha, var_max_iter, var_conv):
    """Literal lda-c lda_inference + compute_likelihood (tiny inputs)."""
    K = lb.shape[0]
    N_ = len(words)
    total = sum(counts)
    gam = [alpha + total / K] * K
    dig = [special.digamma(g) for g in gam]
    phi = [[1.0 / K] * K for _ in range(N_)]
    conv, L_old, it = 1.0, 0.0, 0
    while conv > var_conv and (it < var_max_iter or var_max_iter == -1):
        it += 1
        for n in range(N_):
            old = list(phi[n])
            s = 0.0
            for k in range(K):
                phi[n][k] = dig[k] + lb[k, words[n]]
                s = special.log_sum(s, phi[n][k]) if k > 0 else phi[n][k]
            for k in range(K):
                phi[n][k] = math.exp(phi[n][k] - s)
                gam[k] = gam[k] + counts[n] * (phi[n][k] - old[k])
                dig[k] = special.digamma(gam[k])
        gsum = sum(gam)
        dsum = special.digamma(gsum)
        L = math.lgamma(alpha * K) - K * math.lgamma(alpha) - math.lgamma(gsum)
        for k in range(K):
            L += (alpha - 1) * (dig[k] - dsum) + math.lgamma(gam[k]) - (gam[k] - 1) * (dig[k] - dsum)
            for n in range(N_):
                if phi[n][k] > 0:
                    L += counts[n] * (phi[n][k] * ((dig[k] - dsum) - math.log(phi[n][k]) + lb[k, words[n]]))
        conv = (L_old - L) / L_old
        L_old = L
    return gam, L, it


def test_cpu_estep_matches_literal_ldac():
    c = planted_corpus(num_docs=12, num_terms=30, num_topics=3, mean_tokens=8, seed=5)
    K = 4
    rng = np.random.default_rng(0)
    cw = 1.0 / c.num_terms + rng.random((K, c.num_terms))
    lb = np.log(cw / cw.sum(1, keepdims=True))
    r = N.lda_estep_ldac(c.doc_ptr, c.word_idx, c.counts.astype(float), lb, 0.7, 20, float(np.float32(1e-6)), 1, 1)
    for d in range(c.num_docs):
        a, b = c.doc_ptr[d], c.doc_ptr[d + 1]
        g, L, it = _ldac_inference_py(c.word_idx[a:b].tolist(), c.counts[a:b].tolist(), lb, 0.7, 20,
                                      float(np.float32(1e-6)))
        assert np.allclose(r["gamma"][d], g, rtol=1e-12)
        assert r["doc_likelihood"][d] == pytest.approx(L, rel=1e-12)
        assert r["iters"][d] == it


def test_cpu_estep_thread_invariance():
    c = planted_corpus(num_docs=400, num_terms=300, num_topics=5, seed=1)
    rng = np.random.default_rng(0)
    lb = np.log(rng.dirichlet(np.ones(300), size=8))
    outs = [N.lda_estep_ldac(c.doc_ptr, c.word_idx, c.counts.astype(float), lb, 0.5, 20, 1e-6, 4, t) for t in (1, 3, 8)]
    for o in outs[1:]:
        assert np.array_equal(o["class_word"], outs[0]["class_word"]) and o["likelihood"] == outs[0]["likelihood"]
        assert np.array_equal(o["gamma"], outs[0]["gamma"])


def test_jacobi_and_gauss_seidel_reach_the_same_fixed_point():
    c = planted_corpus(num_docs=200, num_terms=100, num_topics=4, mean_tokens=15, seed=2)
    K = 6
    rng = np.random.default_rng(1)
    lb = np.log(rng.dirichlet(np.ones(100), size=K))
    gs = N.lda_estep_ldac(c.doc_ptr, c.word_idx, c.counts.astype(float), lb, 0.3, -1, 1e-12, 1, 4)
    jc = R.estep_jacobi(torch.from_numpy(c.doc_ptr), torch.from_numpy(c.word_idx), torch.from_numpy(c.counts).double(),
                        torch.from_numpy(np.exp(lb).T.copy()), K, 0.3, -1, 1e-12)
    # per-document variational problem is non-convex: compare the corpus objective and most docs
    assert jc["lik"].sum().item() == pytest.approx(gs["likelihood"], rel=2e-3)
    close = np.isclose(jc["gamma"].numpy(), gs["gamma"], rtol=1e-3, atol=1e-2).all(1).mean()
    assert close > 0.8


def test_torch_engine_em_runs_and_is_monotone():
    c = planted_corpus(num_docs=300, num_terms=200, num_topics=4, seed=3)
    eng = LDAEngine(c, 8, LDASettings(em_max_iter=10), backend="torch", device="cpu", seed=0)
    res = eng.run()
    L = [x[0] for x in res.likelihoods]
    assert all(np.diff(L) > -1e-6 * abs(L[0]))
    assert res.em_iterations <= 11 and eng.alpha > 0


def test_cpu_backend_engine_matches_native_estimate(tmp_path):
    c = planted_corpus(num_docs=150, num_terms=120, num_topics=4, seed=4)
    st = LDASettings(em_max_iter=3)
    eng = LDAEngine(c, 5, st, backend="cpu", seed=2)
    res = eng.run()
    assert len(res.likelihoods) == 4 and all(np.isfinite(x[0]) for x in res.likelihoods)


def test_lda_executable(tmp_path):
    exe = os.path.join(os.path.dirname(native.__file__), "..", "_lib", "lda")
    c = planted_corpus(num_docs=60, num_terms=50, num_topics=3, seed=6)
    ldac.write_model_dat(str(tmp_path / "model.dat"), c)
    (tmp_path / "settings.txt").write_text(LDASettings(em_max_iter=4).dumps())
    out = tmp_path / "out"
    r = subprocess.run([exe, "est", "2.5", "5", str(tmp_path / "settings.txt"), "3", str(tmp_path / "model.dat"),
                        "random", str(out)], capture_output=True, text=True, env=dict(os.environ, ONI_THREADS="2"))
    assert r.returncode == 0, r.stderr
    for f in ("000.beta", "000.other", "005.beta", "005.gamma", "final.beta", "final.gamma", "final.other",
              "likelihood.dat", "word-assignments.dat"):
        assert (out / f).exists(), f
    lb, a = ldac.load_model(str(out / "final"))
    assert lb.shape == (5, c.num_terms) and a > 0
    assert len((out / "likelihood.dat").read_text().splitlines()) == 5
    g = ldac.load_gamma(str(out / "final.gamma"))
    assert g.shape == (60, 5)
    # lda inf with the trained model
    r = subprocess.run([exe, "inf", str(tmp_path / "settings.txt"), str(out / "final"), str(tmp_path / "model.dat"),
                        str(tmp_path / "inf")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert ldac.load_gamma(str(tmp_path / "inf-gamma.dat")).shape == (60, 5)


def test_estimate_files_and_exact_resume(tmp_path):
    c = planted_corpus(num_docs=200, num_terms=150, num_topics=4, seed=7)
    st = LDASettings(em_max_iter=12, em_converged=1e-12)
    full = estimate(c, 6, 2.5, st, "random", str(tmp_path / "full"), backend="torch", device="cpu", seed=3)
    with pytest.raises(RuntimeError):
        estimate(c, 6, 2.5, LDASettings(em_max_iter=12, em_converged=1e-12), "random", str(tmp_path / "part"),
                 backend="torch", device="cpu", seed=3, fault_at_iteration=7)
    assert (tmp_path / "part" / "checkpoint.npz").exists()
    resumed = estimate(c, 6, 2.5, LDASettings(em_max_iter=12, em_converged=1e-12), "random", str(tmp_path / "part"),
                       backend="torch", device="cpu", seed=3, resume=True)
    assert resumed.em_iterations == full.em_iterations
    assert (tmp_path / "part" / "likelihood.dat").read_text() == (tmp_path / "full" / "likelihood.dat").read_text()
    assert np.allclose(resumed.gamma, full.gamma, rtol=1e-9)
    assert (tmp_path / "part" / "final.beta").read_text() == (tmp_path / "full" / "final.beta").read_text()


def test_settings_roundtrip(tmp_path):
    s = LDASettings(var_max_iter=30, var_converged=1e-5, em_max_iter=50, em_converged=1e-3, estimate_alpha=False)
    p = tmp_path / "settings.txt"
    p.write_text(s.dumps())
    s2 = LDASettings.load(str(p))
    assert (s2.var_max_iter, s2.em_max_iter, s2.estimate_alpha) == (30, 50, False)
    assert s2.var_converged == s.var_converged


def test_random_ss_counter_generator():
    """lda-c random start from the counter-based generator: deterministic per seed, thread-count
    invariant, 1/V + U[0, 1), distinct seeds differ."""
    N = native.lib()
    a = N.random_ss(5, 1000, 7, threads=1)
    b = N.random_ss(5, 1000, 7, threads=8)
    assert a.shape == (5, 1000) and np.array_equal(a, b)
    assert not np.array_equal(a, N.random_ss(5, 1000, 8))
    u = a - 1.0 / 1000
    assert u.min() >= 0.0 and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.02


def test_word_assignments_final_pass_cpu_backends():
    """The final-pass assignments of the C++ oracle equal an explicit per-document argmax of the phi it
    leaves (lda-c's literal schedule), and the torch backend's Jacobi form assigns every entry."""
    import numpy as np
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.ops import native
    from oni_ml_amd.synth.corpus import planted_corpus
    c = planted_corpus(num_docs=150, num_terms=200, num_topics=4, seed=2)
    eng = LDAEngine(c, 6, LDASettings(em_max_iter=3), backend="cpu", seed=1)
    eng.run()
    z = eng.word_assignments()
    assert z.shape == (c.nnz,) and z.min() >= 0 and z.max() < 6
    lb = np.log(np.maximum(eng.beta.numpy().T, 1e-300))
    # literal lda_inference for one document, then argmax phi: phi_nk ~ exp(dig_k + lb_kw), dig of the
    # gamma after the word's own update -- recompute through the oracle's E-step on that document alone
    z1 = native.lib().lda_assign_ldac(c.doc_ptr[:2] - 0, c.word_idx[:c.doc_ptr[1]], c.counts[:c.doc_ptr[1]].astype(float),
                                      np.ascontiguousarray(lb), eng.alpha, eng.var_max_iter,
                                      eng.settings.var_converged)
    assert np.array_equal(z1, z[:c.doc_ptr[1]])
    t = LDAEngine(c, 6, LDASettings(em_max_iter=3), backend="torch", device="cpu", seed=1)
    t.run()
    zt = t.word_assignments()
    assert zt.shape == (c.nnz,) and zt.min() >= 0 and zt.max() < 6


def test_cphi_window_bounds_cover_corpus_within_budget():
    """c.phi windows of the fp64 engine: contiguous, covering every document, each within the row
    budget unless it is one document longer than the budget."""
    from oni_ml_amd.models.lda.em import cphi_window_bounds
    rng = np.random.default_rng(0)
    L = rng.integers(0, 50, size=2000)
    L[700], L[701] = 5000, 3000
    ptr = np.concatenate([[0], np.cumsum(L)])
    for budget in (60, 2500, 5000, 9000, int(ptr[-1])):
        w = cphi_window_bounds(ptr, budget)
        assert w[0]["d0"] == 0 and w[-1]["d1"] == len(L)
        assert all(a["d1"] == b["d0"] for a, b in zip(w, w[1:]))
        for x in w:
            assert x["e0"] == ptr[x["d0"]] and x["e1"] == ptr[x["d1"]]
            assert x["e1"] - x["e0"] <= budget or x["d1"] - x["d0"] == 1
    assert len(cphi_window_bounds(ptr, int(ptr[-1]))) == 1


def test_parity_gs_updates_mode():
    """gs_updates = -1: the U per K of profiles/r3_precision_parity.md, resolved for every engine."""
    from oni_ml_amd.models.lda.em import parity_gs_updates, resolved_gs_updates
    from oni_ml_amd.models.lda.settings import LDASettings
    assert [parity_gs_updates(k) for k in (20, 32, 50, 52, 100)] == [32, 32, 64, 64, 1024]
    assert resolved_gs_updates(LDASettings(gs_updates=-1), 50) == 64
    assert resolved_gs_updates(LDASettings(gs_updates=0), 50) == 0
    assert resolved_gs_updates(LDASettings(gs_updates=16), 100) == 16


def test_lda_executable_gs_updates(tmp_path):
    """`lda est ... --gs-updates U` runs the GPU engine's block schedule in the C++ baseline: the same
    result as the in-process C++ engine with settings.gs_updates = U; a bad flag is refused."""
    exe = os.path.join(os.path.dirname(native.__file__), "..", "_lib", "lda")
    c = planted_corpus(num_docs=80, num_terms=60, num_topics=3, mean_tokens=60, seed=8)
    ldac.write_model_dat(str(tmp_path / "model.dat"), c)
    (tmp_path / "settings.txt").write_text(LDASettings(em_max_iter=3).dumps())
    outs = {}
    for u in ("0", "4"):
        out = tmp_path / f"out{u}"
        r = subprocess.run([exe, "est", "2.5", "5", str(tmp_path / "settings.txt"), "1", str(tmp_path / "model.dat"),
                            "random", str(out), "--gs-updates", u], capture_output=True, text=True,
                           env=dict(os.environ, ONI_THREADS="2"))
        assert r.returncode == 0, r.stderr
        assert ("block Gauss-Seidel" in r.stdout) == (u != "0")
        outs[u] = (out / "likelihood.dat").read_text()
    assert outs["0"] != outs["4"]          # a different schedule, a different trajectory
    r = subprocess.run([exe, "est", "2.5", "5", str(tmp_path / "settings.txt"), "1", str(tmp_path / "model.dat"),
                        "random", str(tmp_path / "bad"), "--gs-updates", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "usage" in r.stderr


def test_auto_backend_without_gpu_is_ldac_engine():
    """No GPU: backend "auto" is the C++ lda-c engine (csrc/native/lda_ref.cpp), never the Jacobi rehearsal."""
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: auto selects the hip engine")
    c = planted_corpus(num_docs=40, num_terms=30, num_topics=3, seed=9)
    eng = LDAEngine(c, 4, LDASettings(em_max_iter=2), seed=1)
    assert eng.backend == "cpu" and "Gauss-Seidel" in eng.schedule


def test_lda_est_nproc_must_match_world_size(tmp_path):
    """`lda est <nproc>` is oni-lda-c's rank count: a torchrun launch of another size fails loudly."""
    c = planted_corpus(num_docs=30, num_terms=20, num_topics=3, seed=10)
    ldac.write_model_dat(str(tmp_path / "model.dat"), c)
    (tmp_path / "settings.txt").write_text(LDASettings(em_max_iter=2).dumps())
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "lda", "est", "2.5", "4", str(tmp_path / "settings.txt"),
                        "3", str(tmp_path / "model.dat"), "random", str(tmp_path / "o")],
                       capture_output=True, text=True, env=env, cwd=os.path.dirname(os.path.dirname(__file__)))
    assert r.returncode == 1 and "nproc = 3 but 2 ranks" in r.stderr
    r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "lda", "est", "2.5", "4", str(tmp_path / "settings.txt"),
                        "0", str(tmp_path / "model.dat"), "random", str(tmp_path / "o")],
                       capture_output=True, text=True, cwd=os.path.dirname(os.path.dirname(__file__)))
    assert r.returncode == 1 and "nproc must be a positive" in r.stderr
