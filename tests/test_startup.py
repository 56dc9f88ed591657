"""Start-up of a cold ``ml_ops`` process (utils/pycache.py, the fast exit of ``python -m oni_ml_amd``)."""
import importlib.util
import os
import subprocess
import sys

from oni_ml_amd.utils import pycache

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pycache_prefix_only_when_site_packages_read_only(monkeypatch, tmp_path):
    monkeypatch.setattr(sys, "pycache_prefix", None)
    monkeypatch.setenv("XDG_CACHE_HOME", str(tmp_path))
    torch_dir = os.path.dirname(importlib.util.find_spec("torch").origin)
    real = os.access
    # writable installed caches: left alone
    monkeypatch.setattr(os, "access", lambda p, m: True if p.startswith(torch_dir) else real(p, m))
    assert pycache.enable() is None and sys.pycache_prefix is None
    # read-only (the GPU boxes' non-root user): a per-user prefix
    monkeypatch.setattr(os, "access", lambda p, m: False if p.startswith(torch_dir) else real(p, m))
    got = pycache.enable()
    assert got == os.path.join(str(tmp_path), "oni_ml_amd", "pycache") and sys.pycache_prefix == got
    assert os.path.isdir(got)
    # an explicit prefix wins; ONI_PYCACHE=0 disables
    assert pycache.enable() == got
    monkeypatch.setattr(sys, "pycache_prefix", None)
    monkeypatch.setenv("ONI_PYCACHE", "0")
    assert pycache.enable() is None


def test_fast_exit_keeps_outputs(tmp_path):
    """`python -m oni_ml_amd ml_ops` leaves through os._exit after a completed run: the same files,
    byte for byte, as with the full interpreter teardown (ONI_FAST_EXIT=0)."""
    inp = tmp_path / "in"
    env = dict(os.environ, PYTHONPATH=ROOT)
    subprocess.run([sys.executable, "-m", "oni_ml_amd", "synth", "flow", "--out", str(inp) + "/", "--events", "3000"],
                   cwd=ROOT, env=env, check=True, capture_output=True)
    (tmp_path / "none.conf").write_text("")
    outs = {}
    for v in ("1", "0"):
        lp = tmp_path / f"out{v}"
        r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "ml_ops", "20160122", "flow", "1e-3", "--lpath", str(lp),
                            "--flow-path", str(inp), "--conf", str(tmp_path / "none.conf"), "--quiet", "--backend", "cpu"],
                           cwd=ROOT, env=dict(env, ONI_FAST_EXIT=v), capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[v] = {f: (lp / f).read_bytes() for f in ("flow_results.csv", "doc_results.csv", "word_results.csv",
                                                      "final.gamma", "final.beta", "word-assignments.dat")}
    assert outs["1"] == outs["0"]
