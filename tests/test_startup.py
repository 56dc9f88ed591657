"""Start-up of a cold ``ml_ops`` process (utils/pycache.py, the fast exit of ``python -m oni_ml_amd``)."""
import importlib.util
import os
import subprocess
import sys
import time

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
                           cwd=ROOT, env=dict(env, ONI_FAST_EXIT=v, ONI_T_SPAWN=repr(time.time())), capture_output=True,
                           text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        # a timing parent (ONI_T_SPAWN) gets the time of the fast exit call and the memory then resident
        mark = lp / ".exit_mark"
        assert mark.exists() == (v == "1")
        if v == "1":
            t, *kv = mark.read_text().split()
            assert float(t) > 0 and "RssAnon" in dict(x.split("=", 1) for x in kv)
        outs[v] = {f: (lp / f).read_bytes() for f in ("flow_results.csv", "doc_results.csv", "word_results.csv",
                                                      "final.gamma", "final.beta", "word-assignments.dat")}
    assert outs["1"] == outs["0"]


def test_input_prefetch_keeps_outputs(tmp_path):
    """The day's inputs read on a thread while torch imports (pipeline/prefetch.py, ONI_PREFETCH=1, the
    default) give the same files as the load stage reading them itself; the load record says which."""
    import json
    from oni_ml_amd.synth.dns import generate_dns_day
    env = dict(os.environ, PYTHONPATH=ROOT)
    inp = tmp_path / "in"
    subprocess.run([sys.executable, "-m", "oni_ml_amd", "synth", "flow", "--out", str(inp) + "/", "--events", "3000"],
                   cwd=ROOT, env=env, check=True, capture_output=True)
    g = generate_dns_day(str(tmp_path / "dns"), events=4000, seed=3, files=3)
    (tmp_path / "none.conf").write_text("")
    files = {"flow": ("flow_results.csv", "doc_results.csv", "word_results.csv", "final.gamma"),
             "dns": ("dns_results.csv", "doc_results.csv", "word_results.csv", "final.gamma")}
    for src, tol, extra in (("flow", "1e-3", ["--flow-path", str(inp)]),
                            ("dns", "1e-2", ["--dns-path", g["dns_path"], "--top1m", g["top1m"]])):
        outs = {}
        for v in ("1", "0"):
            lp = tmp_path / f"{src}{v}"
            r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "ml_ops", "20160122", src, tol, "--lpath", str(lp),
                                "--conf", str(tmp_path / "none.conf"), "--quiet", "--backend", "cpu"] + extra,
                               cwd=ROOT, env=dict(env, ONI_PREFETCH=v), capture_output=True, text=True, timeout=600)
            assert r.returncode == 0, r.stderr[-2000:]
            recs = [json.loads(x) for x in open(lp / "metrics.jsonl")]
            load = [x for x in recs if x.get("stage") == "load" and x.get("status") == "ok"]
            assert load and load[0]["prefetched"] is (v == "1")
            outs[v] = {f: (lp / f).read_bytes() for f in files[src]}
        assert outs["1"] == outs["0"], src


def test_dns_prefetch_dropped_on_failure(tmp_path):
    """A forked DNS prefetch that no load stage collects (a run failing before its load stage) is killed,
    reaped and its /dev/shm directory removed by prefetch.drop_all (cmd_ml_ops' finally) -- ADVICE r5."""
    from oni_ml_amd.synth.dns import generate_dns_day
    g = generate_dns_day(str(tmp_path / "dns"), events=2000, seed=1, files=2)
    code = f"""
import glob, os
from oni_ml_amd.pipeline import prefetch
before = set(glob.glob('/dev/shm/oni_prefetch_*'))
args = ({g['dns_path']!r}, None, 1000, True, {g['top1m']!r}, 2)
assert prefetch._start_dns_fork(('dns',), args)
(_, box), = prefetch._JOBS.values()
made = set(glob.glob('/dev/shm/oni_prefetch_*')) - before
assert len(made) == 1, made
prefetch.drop_all()
assert not prefetch._JOBS
assert not (set(glob.glob('/dev/shm/oni_prefetch_*')) - before)
try:
    os.waitpid(-1, os.WNOHANG)
    raise SystemExit('a child is left')
except ChildProcessError:
    pass
print('ok')
"""
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]
