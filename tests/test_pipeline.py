"""End-to-end pipelines on the CPU (torch LDA backend): file contract, stage resume, locking, CLI, config."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oni_ml_amd import config as CFG
from oni_ml_amd.models.lda.settings import LDASettings
from oni_ml_amd.pipeline import run
from oni_ml_amd.pipeline.runner import RunLock

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLOW_FILES = ["doc.dat", "words.dat", "model.dat", "final.beta", "final.gamma", "final.other", "likelihood.dat",
              "doc_results.csv", "word_results.csv", "flow_results.csv"]


def _flow_cfg(tmp_path, events=4000, **kw):
    from oni_ml_amd.synth.flow import generate_flow_day
    if not (tmp_path / "in").exists():
        generate_flow_day(str(tmp_path / "in") + "/", events=events, seed=11, n_internal=300, n_external=600)
    cfg = CFG.resolve("20160122", "flow", tol=kw.pop("tol", 1e-3), conf_path=None, environ={},
                      lpath=str(tmp_path / "ml"), flow_path=str(tmp_path / "in"), backend="torch", threads=2,
                      verbose=False, **kw)
    cfg.settings = LDASettings(em_max_iter=3)
    return cfg


def test_flow_pipeline_file_contract(tmp_path):
    cfg = _flow_cfg(tmp_path)
    s = run(cfg, device="cpu", log=lambda *a, **k: None)
    for f in FLOW_FILES:
        assert (tmp_path / "ml" / f).exists(), f
    res = (tmp_path / "ml" / "flow_results.csv").read_text().splitlines()
    assert len(res) == s["scored"] > 0
    keys = []
    for line in res:
        f = line.split(",")
        assert len(f) == 37
        keys.append(min(float(f[35]), float(f[36])))
        assert float(f[35]) < 1e-3 or float(f[36]) < 1e-3
    assert keys == sorted(keys)
    docs = (tmp_path / "ml" / "doc.dat").read_text().splitlines()
    dres = (tmp_path / "ml" / "doc_results.csv").read_text().splitlines()
    assert [d.split(",")[1] for d in docs] == [r.split(",")[0] for r in dres]
    assert len((tmp_path / "ml" / "final.gamma").read_text().splitlines()) == len(docs)
    for r in dres[:20]:
        vals = [float(x) for x in r.split(",")[1].split(" ")]
        assert len(vals) == 20 and abs(sum(vals) - 1) < 1e-9
    wres = (tmp_path / "ml" / "word_results.csv").read_text().splitlines()
    phi = np.array([[float(x) for x in r.split(",")[1].split(" ")] for r in wres])
    assert np.allclose(phi.sum(0), 1.0, atol=1e-8)
    assert all(len(r.split(",")[0]) <= 20 for r in wres)   # strict: S20 truncation
    # metrics.jsonl: stage seconds, the LDA engine's run metrics and the
    # variational-iteration histogram of the last E-step
    recs = [json.loads(l) for l in (tmp_path / "ml" / "metrics.jsonl").read_text().splitlines()]
    lda = [r for r in recs if r.get("stage") == "lda"][-1]
    assert lda["docs_per_sec"] > 0 and lda["var_iter_mean"] >= 1 and lda["exchange"] == "none"
    assert lda["exchange_bytes_per_iter"] == 0 and "schedule" in lda
    det = [r for r in recs if r.get("stage") == "lda_detail"][-1]
    assert sum(det["var_iter_hist"]) == len(docs) and det["var_iter_hist"][0] == 0


def test_flow_pipeline_fixed_mode_and_resume(tmp_path):
    cfg = _flow_cfg(tmp_path, compat="fixed", topics=7)
    run(cfg, device="cpu", log=lambda *a, **k: None)
    first = (tmp_path / "ml" / "flow_results.csv").read_text()
    assert len((tmp_path / "ml" / "doc_results.csv").read_text().splitlines()[0].split(",")[1].split(" ")) == 7
    # resume after lda: only lda_post + flow_post rerun, same results
    os.unlink(tmp_path / "ml" / ".stages" / "lda_post.done")
    os.unlink(tmp_path / "ml" / ".stages" / "flow_post.done")
    os.unlink(tmp_path / "ml" / "flow_results.csv")
    cfg2 = _flow_cfg(tmp_path, compat="fixed", topics=7, resume=True)
    logs = []
    run(cfg2, device="cpu", log=logs.append)
    again = (tmp_path / "ml" / "flow_results.csv").read_text()
    assert again.splitlines() == first.splitlines() if len(first) < 2000 else hash(again) == hash(first)
    assert any("lda] already complete" in l for l in logs)


def test_flow_feedback_changes_corpus_weights(tmp_path):
    from oni_ml_amd.synth.flow import generate_flow_day, generate_flow_feedback
    r = generate_flow_day(str(tmp_path / "in") + "/", events=3000, seed=5, n_internal=200, n_external=300)
    rows = open(r["paths"][0]).read().splitlines()[1:]
    os.makedirs(tmp_path / "ml", exist_ok=True)
    generate_flow_feedback(str(tmp_path / "ml" / "flow_scores.csv"), rows, n=4)
    cfg = _flow_cfg(tmp_path)
    s = run(cfg, device="cpu", log=lambda *a, **k: None)
    assert s["input"]["feedback_rows"] == 4
    counts = [int(tok.split(":")[1]) for line in (tmp_path / "ml" / "model.dat").read_text().splitlines()
              for tok in line.split()[1:]]
    assert max(counts) >= 1000


def test_prefetched_host_cuts_equal_device_rule(tmp_path):
    """The input prefetch's host cuts (pipeline/prefetch.py load_flow_inputs) are bit for bit the stages'
    own ECDF (quantiles.ecdf_cuts): every row weighted (feedback x DUPFACTOR) for flow_pre, the raw rows for
    flow_post; and the pipeline's outputs are the same files with and without them."""
    import torch
    from oni_ml_amd.features import flow as FF
    from oni_ml_amd.pipeline import prefetch
    from oni_ml_amd.synth.flow import generate_flow_day, generate_flow_feedback
    r = generate_flow_day(str(tmp_path / "in") + "/", events=4000, seed=9, n_internal=200, n_external=300)
    rows = open(r["paths"][0]).read().splitlines()[1:]
    os.makedirs(tmp_path / "ml", exist_ok=True)
    generate_flow_feedback(str(tmp_path / "ml" / "flow_scores.csv"), rows, n=5)
    ft = prefetch.load_flow_inputs(str(tmp_path / "in"), str(tmp_path / "ml" / "flow_scores.csv"), 1000, 2)
    assert ft.n_feedback == 5
    dev = FF.featurize(ft, torch.device("cpu"))
    raw = FF.featurize(ft, torch.device("cpu"), raw_only=True)
    for k in ("time", "ibyt", "ipkt"):
        assert ft.host_cuts["all"][k].tobytes() == dev.cuts[k].tobytes(), k
        assert ft.host_cuts["raw"][k].tobytes() == raw.cuts[k].tobytes(), k
    assert any(ft.host_cuts["all"][k].tobytes() != ft.host_cuts["raw"][k].tobytes() for k in ("time", "ibyt", "ipkt"))
    # a month-sized input keeps the device ECDF (HOST_CUT_ROWS)
    lim = prefetch.HOST_CUT_ROWS
    try:
        prefetch.HOST_CUT_ROWS = ft.n - 1
        big = prefetch.load_flow_inputs(str(tmp_path / "in"), str(tmp_path / "ml" / "flow_scores.csv"), 1000, 2)
        assert getattr(big, "host_cuts", None) is None
    finally:
        prefetch.HOST_CUT_ROWS = lim
    # the whole pipeline with the prefetched table (host cuts) and with its own read: the same files
    outs = []
    for tag, use in (("pre", True), ("own", False)):
        lp = tmp_path / tag
        os.makedirs(lp, exist_ok=True)
        import shutil
        shutil.copy(tmp_path / "ml" / "flow_scores.csv", lp / "flow_scores.csv")
        cfg = CFG.resolve("20160122", "flow", tol=1e-2, conf_path=None, environ={}, lpath=str(lp),
                          flow_path=str(tmp_path / "in"), backend="torch", threads=2, verbose=False)
        cfg.settings = LDASettings(em_max_iter=2)
        if use:
            prefetch.start_for(cfg)
        run(cfg, device="cpu", log=lambda *a, **k: None)
        outs.append({f: (lp / f).read_bytes() for f in ("flow_results.csv", "model.dat", "words.dat", "flow_cuts.json")})
    assert outs[0] == outs[1]


def test_dns_pipeline(tmp_path):
    from oni_ml_amd.synth.dns import generate_dns_day
    r = generate_dns_day(str(tmp_path / "in"), events=6000, seed=3, files=3, n_names=800, n_clients=300)
    cfg = CFG.resolve("20160122", "dns", tol=1e-2, conf_path=None, environ={}, lpath=str(tmp_path / "ml"),
                      dns_path=r["dns_path"], top1m=r["top1m"], backend="torch", threads=2, verbose=False)
    cfg.settings = LDASettings(em_max_iter=2)
    s = run(cfg, device="cpu", log=lambda *a, **k: None)
    rows = (tmp_path / "ml" / "dns_results.csv").read_text().splitlines()
    assert len(rows) == s["scored"] > 0
    for line in rows[:50]:
        f = line.split(",")
        assert len(f) == 16
        assert f[14].count("_") == 7 and float(f[15]) < 1e-2
    # strict: path index 1 skipped
    assert s["input"]["rows"] < 6000 * 0.7


def test_run_lock(tmp_path):
    p = str(tmp_path / ".lock")
    with RunLock(p):
        with pytest.raises(RuntimeError):
            RunLock(p).__enter__()
    with RunLock(p):
        pass


def test_duxbay_parser():
    text = """
# site config
NODES=('node01' 'node02')
UINODE='ui01'
LUSER=/home/duxbay
HPATH=${LUSER}/ml/${DSOURCE}/${FDATE}
LPATH=${LUSER}/ml/${FDATE}
FLOW_PATH="/user/duxbay/flow/csv/y=${YR}/m=${MH}/d=${DY}/"
export TOL=1e-20
RAW='${LUSER}'
"""
    d = CFG.parse_duxbay(text, CFG.run_vars("20160122", "flow"))
    assert d["NODES"] == ["node01", "node02"] and d["UINODE"] == "ui01"
    assert d["HPATH"] == "/home/duxbay/ml/flow/20160122"
    assert d["FLOW_PATH"] == "/user/duxbay/flow/csv/y=2016/m=01/d=22/"
    assert d["TOL"] == "1e-20" and d["RAW"] == "${LUSER}"


def test_config_layering(tmp_path):
    conf = tmp_path / "duxbay.conf"
    conf.write_text("LUSER=/data/u\nLPATH=${LUSER}/ml/${FDATE}\nFLOW_PATH=/a\nTOL=1e-5\n")
    c = CFG.resolve("20160122", "flow", conf_path=str(conf), environ={"FLOW_PATH": "/b"})
    assert c.lpath == "/data/u/ml/20160122" and c.flow_path == "/b" and c.tol == 1e-5
    c = CFG.resolve("20160122", "flow", tol=1e-9, conf_path=str(conf), environ={}, topics=30)
    assert c.tol == 1e-9 and c.topics == 30 and c.flow_path == "/a"


def test_cli_syntax_error():
    r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "ml_ops", "2016", "flow"], cwd=ROOT, capture_output=True,
                       text=True)
    assert "ml_ops.sh syntax error" in r.stdout


def test_launcher_environment(tmp_path):
    """scripts/ml_ops.sh (bench.py's cold leg goes through it) execs the package with THP-backed malloc
    (glibc.malloc.hugetlb=1, prepended to any GLIBC_TUNABLES already set) and reports the reference's
    syntax error."""
    shim = tmp_path / "python"
    shim.write_text('#!/bin/bash\necho "TUNABLES=${GLIBC_TUNABLES}"\n')
    shim.chmod(0o755)
    env = dict(os.environ, PATH=f"{tmp_path}:{os.environ['PATH']}", GLIBC_TUNABLES="glibc.malloc.arena_max=2")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "ml_ops.sh"), "20160122", "flow"], env=env,
                       capture_output=True, text=True)
    assert r.stdout.strip() == "TUNABLES=glibc.malloc.hugetlb=1:glibc.malloc.arena_max=2"
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "ml_ops.sh"), "2016", "flow"], capture_output=True,
                       text=True)
    assert "ml_ops.sh syntax error" in r.stdout


def test_cli_end_to_end_and_lda_est(tmp_path):
    from oni_ml_amd.synth.flow import generate_flow_day
    generate_flow_day(str(tmp_path / "in") + "/", events=3000, seed=2, n_internal=200, n_external=300)
    st = tmp_path / "settings.txt"
    st.write_text(LDASettings(em_max_iter=2).dumps())
    env = dict(os.environ, ONI_CONF=str(tmp_path / "none.conf"))
    r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "ml_ops", "20160122", "flow", "1e-3", "--lpath",
                        str(tmp_path / "ml"), "--flow-path", str(tmp_path / "in"), "--backend", "torch", "--settings",
                        str(st), "--threads", "2", "--quiet"], cwd=ROOT, capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    summ = json.load(open(tmp_path / "ml" / "run_summary.json"))
    assert summ["scored"] > 0 and (tmp_path / "ml" / "flow_results.csv").exists()
    assert not (tmp_path / "ml" / "doc_wc.dat").exists()
    # lda est on the produced corpus (GPU engine's CLI, torch backend here)
    r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "lda", "est", "2.5", "20", str(st), "1",
                        str(tmp_path / "ml" / "model.dat"), "random", str(tmp_path / "lda"), "--backend", "torch"],
                       cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "lda" / "final.gamma").exists() and (tmp_path / "lda" / "word-assignments.dat").exists()
    # lda_post on that directory with the reference's file names
    import shutil
    for f in ("doc.dat", "words.dat"):
        shutil.copy(tmp_path / "ml" / f, tmp_path / "lda" / f)
    r = subprocess.run([sys.executable, "-m", "oni_ml_amd", "lda_post", str(tmp_path / "lda") + "/"], cwd=ROOT,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "lda" / "word_results.csv").exists()


def test_hive_ntile_semantics():
    from oni_ml_amd.features.quantiles import hive_ntile_max
    rng = np.random.default_rng(3)
    for N, n in [(100, 10), (101, 10), (7, 3), (2, 10), (1, 3)]:
        v = rng.integers(0, 50, N).astype(float)
        got = hive_ntile_max(v, n)
        # literal ntile: row i (0-based, sorted) goes to tile 1 + i // ceil-ish split
        s = np.sort(v, kind="stable")
        tiles = min(n, N)
        base, extra = divmod(N, tiles)
        tile_of = []
        for t in range(tiles):
            tile_of += [t + 1] * (base + (t < extra))
        want = [(max(s[i] for i in range(N) if tile_of[i] == t), t) for t in range(1, tiles + 1)]
        assert got == want


def test_qtiles_gen_cli_and_fixed_cuts(tmp_path):
    """gen_qtiles.sh + qtiles.py -> flow_qtiles, then a run with those fixed cuts (the CUT consumer)."""
    from oni_ml_amd.cli import main
    from oni_ml_amd.features.quantiles import parse_qtiles
    cfg = _flow_cfg(tmp_path)
    assert main(["qtiles", "gen", cfg.flow_path, "--out", str(tmp_path / "q"), "--keep-tsv"]) == 0
    text = (tmp_path / "q" / "flow_qtiles").read_text()
    q = parse_qtiles(text)
    assert q["ibyt"][0] == 0 and len(q["ibyt"]) == 11 and len(q["ipkt"]) == 4 and len(q["time"]) == 11
    assert all(np.diff(q[k]).min() >= 0 for k in q)
    tsv = (tmp_path / "q" / "qtiles.tsv").read_text().splitlines()
    assert tsv.count("|") == 2 and tsv[0].endswith("\t1")
    cfg.cuts = str(tmp_path / "q" / "flow_qtiles")
    run(cfg, device="cpu", log=lambda *a, **k: None)
    saved = json.loads((tmp_path / "ml" / "flow_cuts.json").read_text())["cuts"]
    for k in ("ibyt", "ipkt", "time"):
        assert saved[k] == q[k].tolist()


def test_cut_environment_variable():
    c = CFG.resolve("20160122", "flow", conf_path=None, environ={"CUT": "0 10 20,0 1,0 5.5", "FLOW_PATH": "/x",
                                                                   "LPATH": "/y"})
    assert c.fixed_cuts()["time"].tolist() == [0.0, 5.5]


def test_install_dry_run(tmp_path, capsys):
    from oni_ml_amd.cli import main
    conf = tmp_path / "duxbay.conf"
    conf.write_text('NODES=(node01 node02)\nLUSER=/home/oni\n')
    assert main(["install", "--conf", str(conf), "--dry-run"]) == 0
    out = capsys.readouterr().out.splitlines()
    assert len(out) == 2 and out[0].startswith("rsync -v -a --exclude=.* ") and out[1].endswith("node02:/home/oni/ml")


def test_hdfs_hooks_command_sequence(tmp_path):
    from oni_ml_amd.io.hdfs import Hdfs
    calls = []
    h = Hdfs("hadoop", runner=lambda cmd: calls.append(cmd))
    local = h.stage_inputs("hdfs://nn/flow/2016/01/22,/local/x", str(tmp_path / "st"))
    assert local.split(",")[1] == "/local/x" and local.split(",")[0].endswith("in000")
    assert calls[0][:3] == ["hadoop", "fs", "-copyToLocal"] and calls[0][3] == "hdfs://nn/flow/2016/01/22/*"
    calls.clear()
    h.publish("/lp", "/hp", "flow")
    flat = [" ".join(c[2:]) for c in calls]
    assert flat == ["-rm /hp/doc_results.csv", "-put /lp/doc_results.csv /hp/.", "-rm /hp/word_results.csv",
                    "-put /lp/word_results.csv /hp/.", "-rm -R -f /hp/word_counts", "-rm -R -f /hp/scored",
                    "-mkdir -p /hp/scored", "-put /lp/flow_results.csv /hp/scored/part-00000"]


def test_stage_runner_deferred_markers(tmp_path):
    """A stage whose files are written in the background is marked complete only after its writer
    finished; a failed writer raises StageFailed at finish_deferred and leaves no marker."""
    from oni_ml_amd.pipeline.runner import StageFailed, StageRunner
    R = StageRunner(str(tmp_path), resume=True, log=lambda *a, **k: None)
    done = []
    with R.stage("a") as res:
        res["_defer"] = lambda: done.append(1)
    assert not R.done("a")                     # marker waits for the files
    with R.stage("b"):
        pass
    assert R.done("b")
    R.finish_deferred()
    assert done == [1] and R.done("a")

    def boom():
        raise OSError("disk full")
    with R.stage("c") as res:
        res["_defer"] = boom
    with pytest.raises(StageFailed):
        R.finish_deferred()
    assert not R.done("c")
    with R.stage("d") as res:
        res["_defer"] = boom
    R.finish_deferred(suppress=True)           # another error already propagating
    assert not R.done("d")


def test_background_writer_join_reraises():
    """pipeline/common.py background(): the join callable a stage defers re-raises the thread's error."""
    from oni_ml_amd.pipeline import common as C
    out = []
    C.background(lambda: out.append(1))()
    assert out == [1]

    def boom():
        raise OSError("disk full")
    join = C.background(boom)
    with pytest.raises(OSError, match="disk full"):
        join()


@pytest.mark.parametrize("compat", ["strict", "fixed"])
def test_flow_post_paths_byte_identical(tmp_path, monkeypatch, compat):
    """The big-table paths of the one-process flow pipeline write the bytes of the plain ones: the
    deferred lda_post text (on from pipeline/common.py DEFER_POST_VALUES values) and, in fixed mode, the
    scorer's key -> φ row map instead of the word-name dictionary (checked against a resumed run,
    which scores through the names as written)."""
    outs = {}
    from oni_ml_amd.pipeline import common as PC
    for tag, limit in (("plain", 1 << 62), ("deferred", 0)):
        monkeypatch.setattr(PC, "DEFER_POST_VALUES", limit)
        d = tmp_path / tag
        d.mkdir()
        cfg = _flow_cfg(d, compat=compat)
        s = run(cfg, device="cpu", log=lambda *a, **k: None)
        assert s["scored"] > 0
        outs[tag] = {f: (d / "ml" / f).read_bytes() for f in FLOW_FILES}
    assert outs["plain"] == outs["deferred"]
    # a resumed flow_post (tables from the result files, no vocabulary keys): the same flow_results.csv
    d = tmp_path / "deferred"
    os.unlink(d / "ml" / ".stages" / "flow_post.done")
    os.unlink(d / "ml" / "flow_results.csv")
    cfg = _flow_cfg(d, compat=compat)
    cfg.resume = True
    run(cfg, device="cpu", log=lambda *a, **k: None)
    assert (d / "ml" / "flow_results.csv").read_bytes() == outs["plain"]["flow_results.csv"]
