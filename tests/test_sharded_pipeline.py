"""Row-sharded ml_ops pipeline (pipeline/sharded.py) over 2, 4 and 8 gloo ranks == one process, byte for
byte: every file of the run (corpus files, doc_wc.dat, the lda-c model files, doc_results.csv,
word_results.csv and the scored results).

ONI_DIST_DETERMINISTIC=chain makes the LDA model itself independent of the number of ranks (the
sufficient statistics and likelihood sums are one sequential fold over the documents in corpus
order, continued rank after rank), so any difference in the files is a sharding error of the
featurization, corpus builder, export or scoring stages."""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_dist import _free_port  # noqa: E402

FLOW_FILES = ["words.dat", "doc.dat", "model.dat", "doc_wc.dat", "final.beta", "final.gamma", "final.other",
              "likelihood.dat", "005.gamma", "word-assignments.dat", "doc_results.csv", "word_results.csv",
              "flow_results.csv", "flow_cuts.json"]
DNS_FILES = ["words.dat", "doc.dat", "model.dat", "doc_wc.dat", "final.beta", "final.gamma", "likelihood.dat",
             "doc_results.csv", "word_results.csv", "dns_results.csv"]


def _cfg(kind, indir, lpath, extra):
    from oni_ml_amd import config as CFG
    from oni_ml_amd.models.lda.settings import LDASettings
    kw = dict(flow_path=indir) if kind == "flow" else dict(dns_path=extra["dns_path"], top1m=extra["top1m"])
    cfg = CFG.resolve("20160122", kind, tol=extra["tol"], conf_path=None, environ={}, lpath=lpath, backend="torch",
                      threads=2, verbose=False, **kw)
    cfg.settings = LDASettings(em_max_iter=6)
    if extra.get("compat"):
        cfg.compat = extra["compat"]
    cfg.resume = bool(extra.get("resume"))
    return cfg


def _worker(rank, world, port, kind, indir, lpath, extra, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), ONI_DIST_DETERMINISTIC="chain")
    torch.set_num_threads(1)
    try:
        from oni_ml_amd.parallel import dist as D
        from oni_ml_amd.pipeline import run
        ctx = D.init_from_env(backend="gloo")
        s = run(_cfg(kind, indir, lpath, extra), dist=ctx if world > 1 else None, device="cpu",
                log=lambda *a, **k: None)
        q.put((rank, s.get("scored")))
        ctx.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def _run(world, kind, indir, lpath, extra):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, kind, indir, lpath, extra, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=600) for _ in ps], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    for r, o in out:
        assert not isinstance(o, str), o
    return out


@pytest.fixture(scope="module")
def flow_day(tmp_path_factory):
    from oni_ml_amd.synth.flow import generate_flow_day, generate_flow_feedback
    d = tmp_path_factory.mktemp("shflow")
    generate_flow_day(str(d / "in") + "/", events=5000, seed=3, n_internal=300, n_external=700, files=3)
    rows = (d / "in" / "part-00000.csv").read_text().splitlines()[1:300]
    generate_flow_feedback(str(d / "fb.csv"), rows, seed=2, n=12)
    return d


@pytest.mark.parametrize("compat", ["strict", "fixed"])
def test_sharded_flow_pipeline_bytes_equal_one_process(flow_day, compat, tmp_path):
    extra = dict(tol=1e-3, compat=compat)
    one = tmp_path / "w1"
    one.mkdir()
    os.link(flow_day / "fb.csv", one / "flow_scores.csv")
    r1 = _run(1, "flow", str(flow_day / "in"), str(one), extra)
    assert r1[0][1] > 0
    for world in (2, 4, 8):     # 8: the ranks of one MI355X node (the reference's job: 20 MPI ranks)
        lp = tmp_path / f"w{world}"
        lp.mkdir()
        os.link(flow_day / "fb.csv", lp / "flow_scores.csv")
        rn = _run(world, "flow", str(flow_day / "in"), str(lp), extra)
        assert all(o == r1[0][1] for _, o in rn)
        for f in FLOW_FILES:
            a, b = (one / f).read_bytes(), (lp / f).read_bytes()
            assert a == b, (world, f, len(a), len(b))
        # no part files left behind
        assert not [p for p in os.listdir(lp) if ".part" in p]
        # every rank ran every stage (per-rank stage times in metrics.rank<r>.jsonl)
        import json
        for r in range(1, world):
            recs = [json.loads(l) for l in (lp / f"metrics.rank{r}.jsonl").read_text().splitlines()]
            ran = {x["stage"] for x in recs if x.get("status") == "ok"}
            assert {"load", "flow_pre", "lda_pre", "lda", "lda_post", "flow_post"} <= ran, ran


@pytest.mark.parametrize("world,after", [(2, "lda_pre"), (3, "lda_pre"), (3, "lda")])
def test_sharded_flow_resume_bytes_equal_one_process(flow_day, world, after, tmp_path):
    """A sharded run resumed after lda_pre (the lda stage reloads the corpus files on every rank, the
    engine shards them by its own rule) or after lda (gamma sliced from final.gamma, the scorers index
    the document rows through doc_results.csv) writes the files of an uninterrupted one-process run."""
    extra = dict(tol=1e-3, compat="fixed")
    one = tmp_path / "w1"
    one.mkdir()
    os.link(flow_day / "fb.csv", one / "flow_scores.csv")
    r1 = _run(1, "flow", str(flow_day / "in"), str(one), extra)
    lp = tmp_path / f"w{world}"
    lp.mkdir()
    os.link(flow_day / "fb.csv", lp / "flow_scores.csv")
    _run(world, "flow", str(flow_day / "in"), str(lp), extra)
    later = ["lda", "lda_post", "flow_post"][(1 if after == "lda" else 0):]
    outputs = {"lda": ["final.beta", "final.gamma", "final.other", "likelihood.dat", "word-assignments.dat"],
               "lda_post": ["doc_results.csv", "word_results.csv"], "flow_post": ["flow_results.csv"]}
    for st in later:
        os.unlink(lp / ".stages" / f"{st}.done")
        for f in outputs[st]:
            os.unlink(lp / f)
    rn = _run(world, "flow", str(flow_day / "in"), str(lp), dict(extra, resume=True))
    assert all(o == r1[0][1] for _, o in rn)
    for f in FLOW_FILES:
        a, b = (one / f).read_bytes(), (lp / f).read_bytes()
        assert a == b, (world, after, f, len(a), len(b))


def _dns_feedback(path, dns_path, n=10):
    """dns_scores.csv (24 columns, dns_pre_lda.scala:84-117) with severity 3 on n queries of the day."""
    import pyarrow.parquet as pq
    t = pq.read_table(dns_path.split(",")[0]).to_pylist()[:3 * n]
    lines = [",".join(f"c{i}" for i in range(24))]
    for i, r in enumerate(t):
        f = ["x"] * 24
        f[0], f[23], f[1], f[2], f[3] = str(r["frame_time"]), str(r["unix_tstamp"]), str(r["frame_len"]), \
            str(r["ip_dst"]), str(r["dns_qry_name"])
        f[4], f[5], f[6] = str(r["dns_qry_class"]), str(r["dns_qry_type"]), str(r["dns_qry_rcode"])
        f[18] = "3" if i % 3 else "1"
        if "," not in ",".join(f[:4]) and f[3] != "None":
            lines.append(",".join(f))
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


@pytest.mark.parametrize("compat", ["strict", "fixed"])
def test_sharded_dns_pipeline_bytes_equal_one_process(compat, tmp_path):
    from oni_ml_amd.synth.dns import generate_dns_day
    g = generate_dns_day(str(tmp_path / "in"), events=6000, seed=4, files=4, n_names=700, n_clients=250)
    extra = dict(tol=1e-2, compat=compat, dns_path=g["dns_path"], top1m=g["top1m"])
    outs = {}
    for world in (1, 2, 4, 8):
        lp = tmp_path / f"w{world}"
        lp.mkdir()
        _dns_feedback(str(lp / "dns_scores.csv"), g["dns_path"])
        outs[world] = _run(world, "dns", None, str(lp), extra)
    assert outs[1][0][1] > 0
    for world in (2, 4, 8):
        assert all(o == outs[1][0][1] for _, o in outs[world])
        for f in DNS_FILES:
            a, b = (tmp_path / "w1" / f).read_bytes(), (tmp_path / f"w{world}" / f).read_bytes()
            assert a == b, (world, f, len(a), len(b))
