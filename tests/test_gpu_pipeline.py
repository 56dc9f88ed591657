"""GPU (gfx950) end-to-end: HIP featurization/scoring kernels and the pipelines on cuda:0."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oni_ml_amd import config as CFG
from oni_ml_amd.models.lda.settings import LDASettings
from oni_ml_amd.ops import reference as R

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flow_words_kernel_bitwise(hip):
    rng = np.random.default_rng(0)
    n = 200_000
    ports = np.array([0, 1, 22, 53, 80, 443, 1023, 1024, 1025, 8080, 49152, 65535], np.float64)
    cols = [rng.integers(0, 24, n) * 1.0, rng.integers(0, 60, n) * 1.0, rng.integers(0, 60, n) * 1.0,
            rng.choice(ports, n), rng.choice(ports, n), rng.integers(1, 100, n) * 1.0, rng.integers(28, 9000, n) * 1.0]
    cuts = [torch.tensor([0.0, 2.3, 4.78, 7.41, 9.68, 12.0, 14.2, 16.6, 19.1, 21.6], dtype=torch.float64),
            torch.tensor([0.0, 52, 76, 104, 152, 207, 293, 573, 1234, 3569], dtype=torch.float64),
            torch.tensor([0.0, 1, 1, 2, 4], dtype=torch.float64)]
    g = hip.flow_words(*[torch.from_numpy(c).cuda() for c in cols], *[c.cuda() for c in cuts])
    r = R.flow_words(*[torch.from_numpy(c) for c in cols], *cuts)
    for k in ("time", "time_bin", "ibyt_bin", "ipkt_bin", "word_port", "src_prefix", "dst_prefix"):
        assert torch.equal(g[k].cpu(), r[k]), k


def _flow(tmp_path, backend, device, events=20000, topics=20, gs_updates=0):
    from oni_ml_amd.pipeline import run
    from oni_ml_amd.synth.flow import generate_flow_day
    if not (tmp_path / "in").exists():
        generate_flow_day(str(tmp_path / "in") + "/", events=events, seed=4, n_internal=1500, n_external=3000)
    lp = tmp_path / f"ml_{backend}"
    cfg = CFG.resolve("20160122", "flow", tol=1e-4, conf_path=None, environ={}, lpath=str(lp),
                      flow_path=str(tmp_path / "in"), backend=backend, threads=4, verbose=False, topics=topics)
    cfg.settings = LDASettings(em_max_iter=6)
    cfg.settings.gs_updates = gs_updates
    return run(cfg, device=device, log=lambda *a, **k: None), lp


def test_flow_pipeline_gpu_matches_cpu_path(tmp_path):
    """The whole flow pipeline on the GPU (fp64 block Gauss-Seidel engine) against the CPU path with
    the C++ engine on the same schedule: identical corpus files, the same likelihood trajectory."""
    s_gpu, lg = _flow(tmp_path, "hip", "cuda")
    s_cpu, lc = _flow(tmp_path, "cpu", "cpu", gs_updates=32)
    for f in ("doc.dat", "words.dat", "model.dat"):   # featurization + corpus identical on both devices
        assert (lg / f).read_text() == (lc / f).read_text(), f
    Lg = [float(l.split()[0]) for l in (lg / "likelihood.dat").read_text().splitlines()]
    Lc = [float(l.split()[0]) for l in (lc / "likelihood.dat").read_text().splitlines()]
    assert len(Lg) == len(Lc) and np.allclose(Lg, Lc, rtol=1e-9)
    fg = [l.split(",")[:27] for l in (lg / "flow_results.csv").read_text().splitlines()]
    fc = [l.split(",")[:27] for l in (lc / "flow_results.csv").read_text().splitlines()]
    sg, sc = set(map(tuple, fg)), set(map(tuple, fc))
    assert len(sg) > 0 and len(sg & sc) / max(len(sg | sc), 1) > 0.9


def test_dns_pipeline_gpu(tmp_path):
    from oni_ml_amd.pipeline import run
    from oni_ml_amd.synth.dns import generate_dns_day
    r = generate_dns_day(str(tmp_path / "in"), events=30000, seed=1, files=2)
    cfg = CFG.resolve("20160122", "dns", tol=1e-3, conf_path=None, environ={}, lpath=str(tmp_path / "ml"),
                      dns_path=r["dns_path"], top1m=r["top1m"], backend="hip", threads=4, verbose=False)
    cfg.settings = LDASettings(em_max_iter=5)
    s = run(cfg, device="cuda", log=lambda *a, **k: None)
    rows = (tmp_path / "ml" / "dns_results.csv").read_text().splitlines()
    assert len(rows) == s["scored"] and all(len(l.split(",")) == 16 for l in rows[:100])


def test_hip_estimate_resume_exact(tmp_path):
    from oni_ml_amd.models.lda.estimate import estimate
    from oni_ml_amd.synth.corpus import planted_corpus
    c = planted_corpus(num_docs=3000, num_terms=800, num_topics=6, seed=2)
    st = lambda: LDASettings(em_max_iter=11, em_converged=1e-12)
    full = estimate(c, 20, 2.5, st(), "random", str(tmp_path / "a"), backend="hip", device="cuda", seed=5)
    with pytest.raises(RuntimeError):
        estimate(c, 20, 2.5, st(), "random", str(tmp_path / "b"), backend="hip", device="cuda", seed=5,
                 fault_at_iteration=6)
    res = estimate(c, 20, 2.5, st(), "random", str(tmp_path / "b"), backend="hip", device="cuda", seed=5, resume=True)
    assert (tmp_path / "a" / "likelihood.dat").read_text() == (tmp_path / "b" / "likelihood.dat").read_text()
    assert np.array_equal(res.gamma, full.gamma)


def test_bench_smoke():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--events", "200000",
                        "--converge", "0", "--e2e", "0", "--e2e-cold", "0"], cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 1 and out["value"] > 0 and out["steps"] == 3


def test_lda_inf_hip_matches_references():
    """`lda inf` (held-out documents under a fixed model) on the GPU engine: the fp64 engine against the
    C++ engine with the same schedule (32 refreshes per sweep), and against literal lda-c at the
    corpus-likelihood level."""
    from oni_ml_amd.models.lda.inference import infer
    from oni_ml_amd.models.lda.settings import LDASettings
    c, lb = _inf_case()
    ldac = LDASettings()                                             # lda-c defaults: 20 sweeps, 1e-6
    g64, l64 = infer(c, lb, 0.8, ldac, backend="hip", device="cuda")
    ldac32 = LDASettings()
    ldac32.gs_updates = 32
    g32, l32 = infer(c, lb, 0.8, ldac32, backend="cpu")
    assert np.allclose(l64, l32, rtol=1e-10, atol=1e-9)
    assert np.allclose(g64, g32, rtol=1e-10, atol=1e-12)
    _, l_cpu = infer(c, lb, 0.8, ldac, backend="cpu")
    assert abs(l64.sum() - l_cpu.sum()) / abs(l_cpu.sum()) < 1e-4


def _inf_case():
    from oni_ml_amd.synth.corpus import planted_corpus
    c = planted_corpus(num_docs=400, num_terms=300, num_topics=6, mean_tokens=40, seed=11)
    rng = np.random.default_rng(2)
    b = rng.random((12, 300)) ** 3 + 1e-3
    return c, np.log(b / b.sum(1, keepdims=True))


@pytest.mark.parametrize("conv", [1e-12, 3e-4])
def test_lag_saves_from_snapshots_match_draining_loop(tmp_path, monkeypatch, conv):
    """LAG saves from on-device snapshots with one batch queued ahead (LDAEngine._em_with_snapshots) write
    the same files, byte for byte, as the loop that drains the device at every LAG boundary: the %03d
    models, the checkpoint's statistics, likelihood.dat, final.* (conv 3e-4: the device loop stops before
    the last boundary, which then saves nothing)."""
    from oni_ml_amd.models.lda import em as EM
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.estimate import estimate
    from oni_ml_amd.synth.corpus import planted_corpus
    c = planted_corpus(num_docs=3000, num_terms=800, num_topics=6, seed=4)
    out = {}
    # snap / drain: the LAG state handed to the writer threads as device copies (LDAEngine.save_handoff);
    # pinned: the round-5 path (pinned host copies queued by the EM loop itself)
    for mode in ("snap", "drain", "pinned"):
        if mode == "drain":
            monkeypatch.setattr(LDAEngine, "_snapshot_saves_ok", lambda self: False)
        if mode == "pinned":
            monkeypatch.setattr(LDAEngine, "save_handoff", lambda self, *a, **k: None)
            monkeypatch.setattr(EM._Snapshot, "save_handoff", lambda self, *a, **k: None)
        st = LDASettings(em_max_iter=23, em_converged=conv)
        st.lag = 3
        d = tmp_path / mode
        res = estimate(c, 20, 2.5, st, "random", str(d), backend="hip", device="cuda", seed=5)
        files = sorted(p.name for p in d.iterdir() if p.is_file() and p.suffix not in (".json", ".npz"))
        npz = {p.name: dict(np.load(p)) for p in d.iterdir() if p.suffix == ".npz"}   # (zip entries carry times)
        out[mode] = (res.em_iterations, {f: (d / f).read_bytes() for f in files}, npz)
    for other in ("drain", "pinned"):
        (n1, f1, c1), (n2, f2, c2) = out["snap"], out[other]
        assert n1 == n2 and sorted(f1) == sorted(f2)
        assert any(f.endswith(".beta") and f[:3].isdigit() and f != "000.beta" for f in f1)
        for f in f1:
            assert f1[f] == f2[f], (other, f)
        assert sorted(c1) == sorted(c2) and "checkpoint.npz" in c1
        for name in c1:
            assert sorted(c1[name]) == sorted(c2[name]) and \
                all(np.array_equal(c1[name][k], c2[name][k]) for k in c1[name]), (other, name)
