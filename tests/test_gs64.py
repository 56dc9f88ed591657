"""fp64 block Gauss-Seidel engine (csrc/hip/lda_gs64.hip) against the C++ lda-c oracle.

The oracle is csrc/native/lda_ref.cpp's lda_inference with the same schedule parameter
(gs_updates = U: gamma / digamma refreshed after every chunk of ceil(n / U) words; U >= n is
lda-c's literal per-word schedule).  Both compute in double, so gamma, the per-document
likelihoods, class_word and alpha_ss agree to ~1e-12 relative; the tests pin 1e-10.
"""
import numpy as np
import pytest
import torch

from oni_ml_amd.corpus.csr import Corpus
from oni_ml_amd.models.lda.em import LDAEngine
from oni_ml_amd.models.lda.settings import LDASettings
from oni_ml_amd.ops import native
from oni_ml_amd.synth.corpus import planted_corpus

pytestmark = pytest.mark.gpu


def _edge_corpus(seed, V=1500, D=900, max_len=9000):
    """Every length bucket (tiny / wave / 4-wave / 16-wave), empty documents, duplicated
    (doc, word) entries, counts > 1 and words that never occur."""
    rng = np.random.default_rng(seed)
    lens = np.minimum(rng.zipf(1.4, D), max_len)
    lens[rng.choice(D, 25, replace=False)] = 0
    lens[:3] = [max_len, 3000, 700]
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = rng.integers(0, V - 100, int(ptr[-1]))
    for d in rng.choice(np.flatnonzero(lens > 3), 40, replace=False):
        words[ptr[d] + 1] = words[ptr[d]]
    counts = rng.integers(1, 4, words.size)
    return Corpus(ptr.astype(np.int64), words.astype(np.int32), counts.astype(np.int64), V)


def _log_beta(V, K, seed):
    rng = np.random.default_rng(seed)
    b = rng.random((K, V)) ** 3 + 1e-4
    b[:, -3:] = 0.0                                   # words with class_word == 0: the -100 floor
    lb = np.where(b > 0, np.log(np.where(b > 0, b, 1.0)) - np.log(b.sum(1, keepdims=True)), -100.0)
    return lb


def _oracle(c, lb, alpha, st, U):
    N = native.lib()
    return N.lda_estep_ldac(c.doc_ptr, c.word_idx, c.counts.astype(np.float64), np.ascontiguousarray(lb), alpha,
                            st.var_max_iter, st.var_converged, 1, 0, gs_updates=U)


def _gpu_estep(c, K, lb, alpha, st, U, **kw):
    st.gs_updates = U
    eng = LDAEngine(c, K, st, backend="hip", seed=0, precision="fp64", **kw)
    eng.init_from_model(lb, alpha)
    sc = eng.e_step()
    torch.cuda.synchronize()
    return eng, sc.cpu().numpy()


def _rel(a, b, floor):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), floor)))


@pytest.mark.parametrize("K,U,vconv", [(20, 32, -1e30), (20, 8, -1e30), (3, 32, -1e30), (24, 32, -1e30),
                                       (50, 32, -1e30), (100, 16, -1e30), (128, 32, -1e30), (20, 32, 1e-6),
                                       # U > 32 at K > 32: chunk tables in the c.phi rows, no split kernel
                                       (50, 64, -1e30), (100, 256, -1e30), (64, 1024, -1e30), (50, 128, 1e-6),
                                       # U > 32 at K <= 32 (lda-c's per-word schedule at the reference K = 20):
                                       # gs_chain and the GMT topic-group teams with tables in the c.phi rows
                                       (20, 1024, -1e30), (8, 4096, -1e30), (20, 64, -1e30), (24, 1024, 1e-6)])
def test_estep_matches_oracle(K, U, vconv):
    c = _edge_corpus(seed=K + U)
    lb = _log_beta(c.num_terms, K, seed=K)
    st = LDASettings(var_max_iter=6, var_converged=vconv)
    alpha = 0.37
    ref = _oracle(c, lb, alpha, st, U)
    eng, sc = _gpu_estep(c, K, lb, alpha, LDASettings(var_max_iter=6, var_converged=vconv), U)
    it = eng.iters.cpu().numpy()
    # empty documents: L = lnG(Ka) - K lnG(a) - lnG(Ka) + K lnG(a) is 0 up to the rounding of two
    # different lgamma implementations, so lda-c's (L_old - L) / L_old test (0/0 = NaN stops, +-inf
    # does not) may take 1 or 2+ sweeps; gamma = alpha and L ~ 0 either way
    full = np.diff(c.doc_ptr) > 0
    if vconv < 0:
        assert np.array_equal(it[full], ref["iters"][full])
        same = np.ones(c.num_docs, bool)
    else:
        # a document whose convergence test sits within rounding of 1e-6 may stop one sweep apart
        same = (it == ref["iters"]) | ~full
        assert same.mean() > 0.995, same.mean()
    g = eng.gamma[:, :K].cpu().numpy()
    assert _rel(g[same], ref["gamma"][same], 1e-12) < 1e-10
    lik = eng.lik.cpu().numpy()
    assert _rel(lik[same], ref["doc_likelihood"][same], 1.0) < 1e-10
    if vconv < 0:
        cw = eng._cw_local[:, :K].cpu().numpy()
        cw_ref = np.ascontiguousarray(ref["class_word"].T)
        assert _rel(cw, cw_ref, 1e-30) < 1e-10
        assert np.all(cw[-100:] == 0)                              # words that never occur
        assert abs(sc[0] - ref["likelihood"]) / abs(ref["likelihood"]) < 1e-11
        assert abs(sc[1] - ref["alpha_ss"]) / abs(ref["alpha_ss"]) < 1e-10
        ct = eng.class_total[:K].cpu().numpy()
        assert _rel(ct, ref["class_total"], 1e-30) < 1e-11
    if eng.KS > K:
        assert eng.gamma[:, K:].abs().max().item() == 0


def test_literal_schedule_is_ldac():
    """U >= every document length: the fp64 engine runs lda-c's per-word schedule (oracle U = 0)."""
    c = planted_corpus(num_docs=600, num_terms=400, num_topics=5, mean_tokens=8, tail=3.0, max_tokens=30, seed=5)
    assert c.lengths().max() <= 32
    K, alpha = 20, 0.9
    lb = _log_beta(c.num_terms, K, seed=1)
    st = LDASettings()
    ref = _oracle(c, lb, alpha, st, 0)
    eng, sc = _gpu_estep(c, K, lb, alpha, LDASettings(), 32)
    same = eng.iters.cpu().numpy() == ref["iters"]
    assert same.mean() > 0.995
    assert _rel(eng.gamma[:, :K].cpu().numpy()[same], ref["gamma"][same], 1e-12) < 1e-10


def test_em_run_matches_cpu_engine():
    """Whole EM runs (M-step, device alpha Newton, device convergence test): fp64 GPU engine vs the
    C++ engine with the same schedule, from the same random init."""
    c = planted_corpus(num_docs=1200, num_terms=900, num_topics=6, mean_tokens=50, tail=1.0, max_tokens=20000,
                       seed=21)
    runs = []
    for backend in ("hip", "cpu"):
        st = LDASettings(em_max_iter=6)
        st.gs_updates = 32
        eng = LDAEngine(c, 20, st, backend=backend, seed=3, precision="fp64")
        r = eng.run()
        runs.append((np.array([x[0] for x in r.likelihoods]), eng.alpha, eng.gather_gamma(), eng.log_beta()))
    (L1, a1, g1, b1), (L2, a2, g2, b2) = runs
    assert L1.shape == L2.shape
    assert np.max(np.abs(L1 - L2) / np.abs(L2)) < 1e-9
    assert abs(a1 - a2) / a2 < 1e-9
    assert _rel(g1, g2, 1e-6) < 1e-6
    assert np.max(np.abs(b1 - b2)) < 1e-6


@pytest.mark.gpu
def test_mstep_refills_staged_rows_bitwise(monkeypatch):
    """The M-step launch refilling the next E-step's staged rows (LDAEngine.stage_fuse, default) gives
    whole EM runs bitwise equal to a gs_stage launch before every E-step, and leaves each staged
    position holding its word's final beta row."""
    rng = np.random.default_rng(5)
    V, D = 6000, 400
    lens = np.minimum(rng.zipf(1.6, D), 120)
    lens[:4] = [5000, 3000, 2500, 2100]
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = np.concatenate([rng.choice(V, n, replace=False) for n in lens]).astype(np.int32)
    c = Corpus(ptr.astype(np.int64), words, rng.integers(1, 4, words.size).astype(np.int64), V)
    runs = {}
    for fuse in ("1", "0"):
        st = LDASettings(em_max_iter=7)
        eng = LDAEngine(c, 20, st, backend="hip", seed=9, precision="fp64")
        eng.stage_fuse = fuse == "1"
        assert eng._stages and bool(eng._fused_stages(eng.gs_plan)) == (fuse == "1")
        r = eng.run()
        runs[fuse] = (np.array([x[0] for x in r.likelihoods]), eng.alpha, eng.gather_gamma(), eng.log_beta())
        if fuse == "1":
            beta = eng.beta.cpu().numpy()
            for stg in eng._stages.values():
                buf = stg.buf.view(-1, 10, 64, 2).cpu().numpy()
                ent, cnt = stg.tile_ent.cpu().numpy(), stg.tile_cnt.cpu().numpy()
                for t in range(len(ent)):
                    got = buf[t].transpose(1, 0, 2).reshape(64, 20)[:cnt[t]]
                    assert np.array_equal(got, beta[words[ent[t]:ent[t] + cnt[t]]])
    (L1, a1, g1, b1), (L0, a0, g0, b0) = runs["1"], runs["0"]
    assert len(L1) >= 3 and np.array_equal(L1, L0) and a1 == a0
    assert np.array_equal(g1, g0) and np.array_equal(b1, b0)


def test_gs64_graph_replay_and_gate():
    """The captured E-step graph replays bit-identically; a set done flag skips every launch."""
    c = _edge_corpus(seed=7, max_len=3000)
    K = 20
    lb = _log_beta(c.num_terms, K, seed=2)
    st = LDASettings(var_max_iter=5)
    eng, _ = _gpu_estep(c, K, lb, 0.5, st, 32)
    g1 = eng.gamma.clone()
    eng.e_step()                  # graph replay
    torch.cuda.synchronize()
    assert torch.equal(g1, eng.gamma)
    eng.gamma.zero_()
    eng._params[4] = 1.0          # PARAM_DONE
    eng._graph.replay()
    torch.cuda.synchronize()
    assert eng.gamma.abs().max().item() == 0


@pytest.mark.parametrize("stage", ["1", "0"])
@pytest.mark.parametrize("head", [
    # longest chunk 938 words: past the two prefetched rounds (7 waves x 64 lanes x 2), streamed remainder
    [30000, 20000, 15000, 9000, 6000, 5000, 4000, 3500, 3000, 2500, 2200, 2100],
    [24000, 20000, 15000, 9000, 6000, 5000, 4000, 3500, 3000, 2500, 2200, 2100],
])
def test_longest_documents_match_oracle(head, stage, monkeypatch):
    """The longest-document kernel (gs_wsteam: word waves + a topic wave) against the oracle, on chunks
    that need both prefetched rounds, with more than 8 team8 documents so the XCD-aware workgroup order
    holds empty slots (GSPlan.isolate_longest); with the staged row copies (GSStage, default) and
    gathering from beta."""
    from oni_ml_amd.ops import hip as H
    monkeypatch.setenv("ONI_GS_STAGE", stage)
    rng = np.random.default_rng(11)
    V, D = 40000, 300
    lens = np.minimum(rng.zipf(1.5, D), 200)
    lens[:12] = head
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = np.concatenate([rng.choice(V, n, replace=False) for n in lens]).astype(np.int32)
    counts = rng.integers(1, 4, words.size)
    c = Corpus(ptr.astype(np.int64), words, counts.astype(np.int64), V)
    K, U = 20, 32
    lb = _log_beta(V, K, seed=4)
    st = LDASettings(var_max_iter=4, var_converged=-1e30)
    ref = _oracle(c, lb, 0.41, st, U)
    eng, sc = _gpu_estep(c, K, lb, 0.41, LDASettings(var_max_iter=4, var_converged=-1e30), U)
    launches = {v: o.cpu().numpy() for v, o in eng.gs_plan.plan}
    assert (launches[H.GS_TEAM8] < 0).any() and launches[H.GS_TEAM8][0] == 0   # placement gaps
    assert len(eng._stages) == (1 if stage == "1" else 0)
    assert np.array_equal(eng.iters.cpu().numpy(), ref["iters"])
    assert _rel(eng.gamma[:, :K].cpu().numpy(), ref["gamma"], 1e-12) < 1e-10
    assert _rel(eng.lik.cpu().numpy(), ref["doc_likelihood"], 1.0) < 1e-10
    cw = eng._cw_local[:, :K].cpu().numpy()
    assert _rel(cw, np.ascontiguousarray(ref["class_word"].T), 1e-30) < 1e-10


def test_staged_rows_bitwise_equal_beta_rows(monkeypatch):
    """Staged rows change where the team8 kernel reads beta, not what it reads: the E-step outputs are
    bitwise those of the gather from beta, and the staged copy holds exactly each position's row."""
    from oni_ml_amd.ops import hip as H
    rng = np.random.default_rng(3)
    V, D = 20000, 120
    lens = np.minimum(rng.zipf(1.5, D), 150)
    lens[:5] = [12000, 7000, 4100, 3000, 2100]
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = np.concatenate([rng.choice(V, n, replace=False) for n in lens]).astype(np.int32)
    c = Corpus(ptr.astype(np.int64), words, rng.integers(1, 4, words.size).astype(np.int64), V)
    K = 20
    lb = _log_beta(V, K, seed=8)
    out = {}
    for stage in ("1", "0"):
        monkeypatch.setenv("ONI_GS_STAGE", stage)
        eng, sc = _gpu_estep(c, K, lb, 0.3, LDASettings(var_max_iter=6, var_converged=-1e30), 32)
        out[stage] = (eng.gamma.cpu().numpy(), eng.cphi.cpu().numpy(), eng.lik.cpu().numpy(), sc)
        if stage == "1":
            (st,) = eng._stages.values()
            buf = st.buf.view(-1, K // 2, 64, 2).cpu().numpy()          # [tile][pair][lane][2]
            beta = eng.beta.cpu().numpy()
            ent, cnt = st.tile_ent.cpu().numpy(), st.tile_cnt.cpu().numpy()
            for t in (0, 1, len(ent) - 1):
                rows = beta[words[ent[t]:ent[t] + cnt[t]]]              # [cnt][KS]
                got = buf[t].transpose(1, 0, 2).reshape(64, K)[:cnt[t]]
                assert np.array_equal(got, rows)
                assert not buf[t].transpose(1, 0, 2).reshape(64, K)[cnt[t]:].any()
    for a, b in zip(out["1"], out["0"]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("K,env,U,gmin", [
    (100, {}, 32, 2),                                                   # default split for KS > 32
    (100, {"ONI_GS_SPLIT_MIN": "4000"}, 32, 2),
    (100, {"ONI_GS_SPLIT_MIN": "4000,g=3,batches=8", "ONI_SPLIT_MAX_BLOCKS": "9"}, 32, 2),
    (20, {"ONI_GS_SPLIT_MIN": "3000,g=5"}, 32, 2),                      # forced on a narrow KS
    (52, {"ONI_GS_SPLIT_MIN": "2500"}, 32, 2),
    (50, {}, 64, 2),                                                    # 64-row LDS tables (KS 52, U = 64)
    (50, {"ONI_GS_SPLIT_MIN": "2500,g=3"}, 48, 2),
    # the single-round gathers: per-column passes up to 16 segments, batched at <= 8
    (100, {"ONI_GS_SPLIT_MIN": "2500,g=16,words=16"}, 32, 9),
    (100, {"ONI_GS_SPLIT_MIN": "2500,g=8,words=16"}, 32, 5),
    (20, {"ONI_GS_SPLIT_MIN": "2500,g=12,words=24"}, 32, 9),
    # the two-phase exchange (reduce-scatter of owned columns + all-gather of the totals) past 16 segments
    (100, {"ONI_GS_SPLIT_MIN": "2500,g=32,words=8"}, 32, 32),
    (100, {"ONI_GS_SPLIT_MIN": "2500,g=64,words=8"}, 32, 64),
    (100, {"ONI_GS_SPLIT_MIN": "2500,words=4"}, 32, 100),              # G > NC: segments owning no column
    (50, {"ONI_GS_SPLIT_MIN": "2500,g=64,words=4"}, 64, 64),
    (50, {"ONI_GS_SPLIT_MIN": "2500,g=32,words=4"}, 64, 32),
])
def test_split_documents_match_oracle(K, env, U, gmin, monkeypatch):
    """gs_split (one document over G workgroups exchanging tagged per-chunk partials) against the
    oracle: every replica runs the same refresh, so gamma / likelihood / class_word match at 1e-10."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(K)
    V, D = 40000, 260
    lens = np.minimum(rng.zipf(1.5, D), 200)
    lens[:7] = [30000, 20000, 12000, 9100, 5000, 3100, 2600]
    lens[9] = 0
    _check_split(K, U, lens, V, env, gmin, rng)


@pytest.mark.parametrize("K,U,g", [(100, 1024, 32), (100, 1024, 64), (50, 64, 64)])
def test_split_wide_u_two_phase_match_oracle(K, U, g, monkeypatch):
    """The two-phase exchange with the chunk tables past LDS (U = 1024, lda-c's per-word schedule at K = 100:
    a 70 k-word document has W = 69 words per chunk, so up to 64 segments) and at K = 50, U = 64."""
    monkeypatch.setenv("ONI_GS_SPLIT_MIN", f"2500,g={g},words=1")
    rng = np.random.default_rng(K + U)
    V, D = 90000, 200
    lens = np.minimum(rng.zipf(1.5, D), 200)
    lens[:4] = [70000, 33000, 9000, 3000]
    _check_split(K, U, lens, V, {"ONI_GS_SPLIT_MIN": "x"}, g, rng)


def _check_split(K, U, lens, V, env, gmin, rng):
    D = lens.size
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = np.concatenate([rng.choice(V, n, replace=False) for n in lens]).astype(np.int32)
    counts = rng.integers(1, 4, words.size)
    c = Corpus(ptr.astype(np.int64), words, counts.astype(np.int64), V)
    lb = _log_beta(V, K, seed=5)
    st = LDASettings(var_max_iter=5, var_converged=-1e30)
    ref = _oracle(c, lb, 0.33, st, U)
    eng, sc = _gpu_estep(c, K, lb, 0.33, LDASettings(var_max_iter=5, var_converged=-1e30), U)
    sp = eng.gs_plan.split
    # (past 64 segments the first document takes most of the co-resident launch)
    assert sp is not None and sp.n_docs >= (4 if "ONI_GS_SPLIT_MIN" in env and gmin <= 32 else 2)
    assert max(sp.segments.values()) >= max(2, gmin), sp.segments
    if "ONI_SPLIT_MAX_BLOCKS" in env:
        assert len(sp.batches) >= 2
    assert int(sum(b["error"].item() for b in sp.batches)) == 0
    full = lens > 0      # the empty document's 0/0 convergence test may stop a sweep apart (see above)
    assert np.array_equal(eng.iters.cpu().numpy()[full], ref["iters"][full])
    assert _rel(eng.gamma[:, :K].cpu().numpy(), ref["gamma"], 1e-12) < 1e-10
    assert _rel(eng.lik.cpu().numpy(), ref["doc_likelihood"], 1.0) < 1e-10
    cw = eng._cw_local[:, :K].cpu().numpy()
    assert _rel(cw, np.ascontiguousarray(ref["class_word"].T), 1e-30) < 1e-10
    assert abs(sc[0] - ref["likelihood"]) / abs(ref["likelihood"]) < 1e-11
    # graph replay: the launch epoch moves on, the tags of the previous launch never match
    g1 = eng.gamma.clone()
    eng.e_step()
    torch.cuda.synchronize()
    assert torch.equal(g1, eng.gamma)


@pytest.mark.parametrize("K,split_min", [(20, None), (100, None), (20, "3000"), (50, "3000")])
def test_suff_split_matches_single_pass(K, split_min, monkeypatch):
    """Early / late sufficient statistics (the early pass overlaps the longest-document bucket, the late
    pass adds its rows first; at KS > 32 one pass per stream plus the combine of the shared words) against
    the single CSC pass: class_word, class totals and likelihood.
    split_min: split documents plus all five length buckets = 6 work items, more than the 4 streams
    (the case where a round-robin stream choice would put a bucket beside the late pass's stream)."""
    if split_min:
        monkeypatch.setenv("ONI_GS_SPLIT_MIN", split_min)
    c = _edge_corpus(seed=3, max_len=9000 if split_min else 5000)
    lb = _log_beta(c.num_terms, K, seed=6)
    out = []
    for mode in ("off", "force"):
        eng, sc = _gpu_estep(c, K, lb, 0.45, LDASettings(var_max_iter=4), 32, suff_split=mode)
        assert (eng._suff_split is None) == (mode == "off")
        if mode == "force" and K > 32:   # KS > 32: one pass per stream, shared words combined after
            assert eng._suff_split["mode"] == "groups" and len(eng._suff_split["groups"]) >= 2
        if split_min:
            assert eng.gs_plan.split is not None and len(eng.gs_plan.plan) + 1 >= (6 if K <= 32 else 5), \
                [v for v, _ in eng.gs_plan.plan]
        eng.e_step()                                   # graph replay of the same launch sequence
        torch.cuda.synchronize()
        out.append((eng._cw_local[:, :K].cpu().numpy(), eng.class_total[:K].cpu().numpy(), sc,
                    eng.gamma.cpu().numpy()))
    (cw0, ct0, sc0, g0), (cw1, ct1, sc1, g1) = out
    assert np.array_equal(g0, g1)
    assert _rel(cw1, cw0, 1e-30) < 1e-13
    assert _rel(ct1, ct0, 1e-30) < 1e-13
    assert abs(sc1[0] - sc0[0]) <= 1e-13 * abs(sc0[0])


def test_device_random_init_matches_native():
    """The fp64 engine's on-device lda-c random start equals the native counter-based generator the CPU
    backends use (same bits), and class_total is its column sum."""
    c = planted_corpus(num_docs=200, num_terms=300, num_topics=4, seed=1)
    eng = LDAEngine(c, 20, LDASettings(), backend="hip", seed=11, precision="fp64")
    eng.init_random()
    torch.cuda.synchronize()
    ref = native.lib().random_ss(20, c.num_terms, 11)
    assert np.array_equal(eng.cw[:, :20].cpu().numpy(), ref.T)
    assert eng.cw[:, 20:].abs().max().item() == 0 if eng.KS > 20 else True
    assert _rel(eng.class_total[:20].cpu().numpy(), ref.sum(1), 1e-30) < 1e-14


@pytest.mark.parametrize("vconv", [-1e30, 1e-6])
def test_final_pass_word_assignments_match_oracle(vconv):
    """word-assignments.dat: run_em's final pass -- a fresh E-step under the final model, then the first
    argmax of each word's phi -- on the GPU (c.phi rows of the document kernels alone) against the C++
    oracle's lda_inference + write_word_assignment with the same schedule."""
    c = _edge_corpus(seed=13, max_len=3000)
    K, U, alpha = 20, 32, 0.6
    lb = _log_beta(c.num_terms, K, seed=7)
    st = LDASettings(var_max_iter=8, var_converged=vconv)
    st.gs_updates = U
    eng = LDAEngine(c, K, st, backend="hip", seed=0, precision="fp64")
    eng.init_from_model(lb, alpha)
    z = eng.word_assignments()
    ref = native.lib().lda_assign_ldac(c.doc_ptr, c.word_idx, c.counts.astype(np.float64), np.ascontiguousarray(lb),
                                       alpha, st.var_max_iter, st.var_converged, gs_updates=U)
    if vconv < 0:
        assert np.array_equal(z, ref)
    else:
        # documents whose convergence test sits within rounding of 1e-6 may stop a sweep apart
        assert (z == ref).mean() > 0.999


@pytest.mark.parametrize("K,split_min", [(20, None), (100, None), (20, "3000"), (50, "3000")])
def test_cphi_windows_match_one_buffer(K, split_min, monkeypatch):
    """c.phi windows (the E-step in contiguous document windows sharing one small c.phi buffer, each
    window's suff-stats added in place) against the one-buffer engine: gamma bitwise (the document
    kernels do not change), class_word / class totals / likelihood to summation order, an EM run's
    trajectory, and the final pass's word assignments."""
    if split_min:
        monkeypatch.setenv("ONI_GS_SPLIT_MIN", split_min)
    c = _edge_corpus(seed=5, max_len=9000)
    lb = _log_beta(c.num_terms, K, seed=9)
    KS = {20: 24, 50: 52}.get(K, 104)
    budget_gb = (c.nnz // 3) * KS * 8 / 2**30          # ~3-4 windows
    out = []
    for gb in (None, budget_gb):
        st = LDASettings(var_max_iter=5)
        st.gs_updates = 32
        eng = LDAEngine(c, K, st, backend="hip", seed=0, precision="fp64", cphi_gb=gb)
        assert (eng._cwin is None) == (gb is None)
        if gb is not None:
            assert len(eng._cwin) >= 3 and eng.cphi.shape[0] < c.nnz
        eng.init_from_model(lb, 0.45)
        sc = eng.e_step().cpu().numpy()
        eng.e_step()                                   # graph replay
        torch.cuda.synchronize()
        z = eng.word_assignments()
        out.append((eng.gamma.cpu().numpy(), eng._cw_local[:, :K].cpu().numpy(), eng.class_total[:K].cpu().numpy(),
                    sc, z))
    (g0, cw0, ct0, sc0, z0), (g1, cw1, ct1, sc1, z1) = out
    assert np.array_equal(g0, g1)
    assert _rel(cw1, cw0, 1e-30) < 1e-13
    assert _rel(ct1, ct0, 1e-30) < 1e-13
    assert abs(sc1[0] - sc0[0]) <= 1e-13 * abs(sc0[0]) and abs(sc1[1] - sc0[1]) <= 1e-13 * abs(sc0[1])
    assert np.array_equal(z0, z1)


def test_cphi_windows_em_run():
    """A whole EM run in c.phi windows tracks the one-buffer run (same iterations, likelihoods to 1e-12)."""
    c = planted_corpus(num_docs=1500, num_terms=900, num_topics=6, mean_tokens=60, tail=1.0, max_tokens=9000,
                       seed=4)
    runs = []
    for gb in (None, (c.nnz // 4) * 24 * 8 / 2**30):
        st = LDASettings(em_max_iter=8)
        eng = LDAEngine(c, 20, st, backend="hip", seed=3, precision="fp64", cphi_gb=gb)
        r = eng.run()
        runs.append((np.array([x[0] for x in r.likelihoods]), eng.alpha))
    (L0, a0), (L1, a1) = runs
    assert L0.shape == L1.shape
    assert np.max(np.abs(L1 - L0) / np.abs(L0)) < 1e-12
    assert abs(a1 - a0) <= 1e-12 * a0


@pytest.mark.parametrize("K,U,split", [(50, 128, False), (100, 64, False), (50, 128, True), (100, 1024, True),
                                       (20, 1024, False), (20, 64, False)])
def test_final_pass_word_assignments_large_u(K, U, split, monkeypatch):
    """The final pass with U > 32 against the oracle: the team kernels keep their chunk tables in the c.phi
    rows (4- and 8-wave teams read E_j from row n0 + 1 before the chunk's rows are overwritten); the split
    kernel past its LDS tables keeps them in a per-segment scratch (gs_splitw GM)."""
    monkeypatch.setenv("ONI_GS_SPLIT_MIN", "2000" if split else "0")
    c = _edge_corpus(seed=17, max_len=6000)
    alpha = 0.6
    lb = _log_beta(c.num_terms, K, seed=3)
    st = LDASettings(var_max_iter=6, var_converged=-1e30)
    st.gs_updates = U
    eng = LDAEngine(c, K, st, backend="hip", seed=0, precision="fp64")
    if split:
        assert eng.gs_plan.split is not None and all(b["tab"] is not None for b in eng.gs_plan.split.batches)
    else:
        assert eng.gs_plan.split is None
    eng.init_from_model(lb, alpha)
    z = eng.word_assignments()
    ref = native.lib().lda_assign_ldac(c.doc_ptr, c.word_idx, c.counts.astype(np.float64), np.ascontiguousarray(lb),
                                       alpha, st.var_max_iter, st.var_converged, gs_updates=U)
    assert np.array_equal(z, ref)


def test_large_u_at_narrow_topics_plans_table_free_kernels():
    """U > 32 at K <= 32 (the opt-in parity mode, --gs-updates up to 4096 at K = 20): no launch of a kernel
    whose chunk tables live in LDS (gs_small, the one-wave team, gs_wteam / gs_wsteam), no staged rows."""
    from oni_ml_amd.ops import hip as H
    c = _edge_corpus(seed=3, max_len=5000)
    for U in (64, 1024, 4096):
        st = LDASettings()
        st.gs_updates = U
        eng = LDAEngine(c, 20, st, backend="hip", seed=0, precision="fp64")
        kinds = {v for v, _ in eng.gs_plan.plan}
        assert kinds <= {H.GS_TINY, H.GS_CHAIN, H.GS_TEAM4, H.GS_TEAM8}, kinds
        assert H.GS_CHAIN in kinds and not eng._stages and eng.gs_plan.split is None
    st = LDASettings()
    st.gs_updates = 4097
    with pytest.raises(ValueError, match="supports 1..4096"):
        LDAEngine(c, 20, st, backend="hip", seed=0, precision="fp64")


@pytest.mark.parametrize("K,xs", [
    (20, dict(docs=3)),                                  # LDS-minimum members, placement-checked stores
    (20, dict(docs=3, proto=0)),                         # write-through stores only
    (20, dict(docs=4, members=11)),                      # more members than the LDS needs
    (8, dict(docs=2, members=3)),                        # > 64 words of a chunk per member
    (32, dict(docs=2)),                                  # one member part per column (KS + 1 = 33)
])
def test_xsplit_documents_match_oracle(K, xs):
    """gs_xsplit (csrc/hip/experimental/lda_xsplit.hip: one document over one-wave members of one XCD, beta rows resident
    in LDS, 16-byte self-tagged granules) against the oracle at 1e-10, every member replaying the same
    refresh; graph replay moves the launch epoch on.  The experimental module is built only on request
    (`python -m oni_ml_amd._build exp`; measured not faster, profiles/r5_xcd_split.md)."""
    from oni_ml_amd.ops import hip as H
    if not H.exp_available():
        pytest.skip("experimental module _onihip_exp not built (python -m oni_ml_amd._build exp)")
    rng = np.random.default_rng(K + 7)
    V, D = 40000, 260
    lens = np.minimum(rng.zipf(1.5, D), 200)
    lens[:6] = [30000, 20000, 12000, 9100, 5000, 3100]
    lens[9] = 0
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = np.concatenate([rng.choice(V, n, replace=False) for n in lens]).astype(np.int32)
    counts = rng.integers(1, 4, words.size)
    c = Corpus(ptr.astype(np.int64), words, counts.astype(np.int64), V)
    lb = _log_beta(V, K, seed=5)
    for vconv in (-1e30, 1e-6):
        st = LDASettings(var_max_iter=5, var_converged=vconv)
        ref = _oracle(c, lb, 0.33, st, 32)
        eng, sc = _gpu_estep(c, K, lb, 0.33, LDASettings(var_max_iter=5, var_converged=vconv), 32, xsplit=xs)
        sp = eng.gs_plan.split
        assert sp is not None and sp.n_docs == xs["docs"]
        (b,) = sp.batches
        assert b.get("x") and int(b["error"].item()) == 0
        if xs.get("proto", 1) == 1:
            assert set(b["placed"].cpu().tolist()) <= {0, 1}
        full = lens > 0
        it = eng.iters.cpu().numpy()
        same = (it == ref["iters"]) | ~full
        if vconv < 0:
            assert same.all()
        else:
            assert same.mean() > 0.99 and same[:6].all()
        assert _rel(eng.gamma[:, :K].cpu().numpy()[same], ref["gamma"][same], 1e-12) < 1e-10
        assert _rel(eng.lik.cpu().numpy()[same], ref["doc_likelihood"][same], 1.0) < 1e-10
        if vconv < 0:
            cw = eng._cw_local[:, :K].cpu().numpy()
            assert _rel(cw, np.ascontiguousarray(ref["class_word"].T), 1e-30) < 1e-10
            assert abs(sc[0] - ref["likelihood"]) / abs(ref["likelihood"]) < 1e-11
            g1 = eng.gamma.clone()
            eng.e_step()
            torch.cuda.synchronize()
            assert torch.equal(g1, eng.gamma)
