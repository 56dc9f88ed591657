"""Row-sharded featurization (features/flow_dist.py) over gloo ranks == one process featurizing all
rows: the same cuts, word space, doc_wc and lda-c corpus (doc.dat / words.dat / model.dat content)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_dist import _free_port  # noqa: E402


def _single(indir, fb, strict=True):
    from oni_ml_amd.corpus.builder import concat, count_pairs, lda_pre
    from oni_ml_amd.features import flow as FF
    ft = FF.load_flow(indir, fb, 1000, threads=3)
    feat = FF.featurize(ft, "cpu")
    ws = FF.word_space_for(feat)
    src, dst = FF.word_keys(feat, ws)
    dwc = concat([count_pairs(feat.sip, src, feat.weight), count_pairs(feat.dip, dst, feat.weight)], merge=not strict)
    b = lda_pre(dwc)
    ipn = ft.ip_names
    return dict(cuts={k: v.tolist() for k, v in feat.cuts.items()}, ports=ws.ports.tolist(),
                docs=[ipn[i] for i in b.doc_keys.tolist()], words=ws.decode(b.word_keys),
                ptr=b.corpus.doc_ptr.tolist(), widx=b.corpus.word_idx.tolist(), cnt=b.corpus.counts.tolist(),
                rows=ft.n)


def _worker(rank, world, port, indir, fb, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    try:
        from oni_ml_amd.corpus.sharded import build_sharded
        from oni_ml_amd.features import flow_dist as FD
        from oni_ml_amd.parallel import dist as D
        ctx = D.init_from_env(backend="gloo")
        ft = FD.load_flow_sharded(ctx, indir, fb, 1000, threads=2)
        sections, names, gmap, ws, cuts = FD.featurize_sharded(ctx, ft, "cpu")
        sc = build_sharded(ctx, sections, len(names))
        c = sc.corpus
        q.put((rank, dict(cuts={k: v.tolist() for k, v in cuts.items()}, ports=ws.ports.tolist(),
                          docs=names.take(sc.doc_keys), words=ws.decode(sc.word_keys),
                          ptr=c.doc_ptr.tolist(), widx=c.word_idx.tolist(), cnt=c.counts.tolist(), rows=ft.n,
                          doc_range=sc.doc_range, bounds=sc.bounds, D=sc.num_docs, nnz=sc.nnz)))
        ctx.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.fixture(scope="module")
def flow_input(tmp_path_factory):
    from oni_ml_amd.synth.flow import generate_flow_day, generate_flow_feedback
    d = tmp_path_factory.mktemp("flowdist")
    generate_flow_day(str(d / "in") + "/", events=6000, seed=5, n_internal=400, n_external=900, files=3)
    rows = (d / "in" / "part-00000.csv").read_text().splitlines()[1:200]
    generate_flow_feedback(str(d / "fb.csv"), rows, seed=1, n=15)
    return str(d / "in"), str(d / "fb.csv")


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_featurization_equals_single_process(flow_input, world):
    indir, fb = flow_input
    ref = _single(indir, fb)
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, indir, fb, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=300) for _ in ps], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    for r, o in out:
        assert isinstance(o, dict), o
    assert sum(o["rows"] for _, o in out) == ref["rows"]          # the byte ranges partition the rows
    from oni_ml_amd.parallel.dist import engine_bounds
    rptr = np.asarray(ref["ptr"])
    want_bounds = [b[0] for b in engine_bounds(rptr, world)] + [len(rptr) - 1]
    for r, o in out:
        for k in ("cuts", "ports", "words"):
            assert o[k] == ref[k], (r, k)
        # each rank holds exactly its engine shard (engine_bounds) of the one-process corpus
        assert o["bounds"] == want_bounds and o["D"] == len(rptr) - 1 and o["nnz"] == rptr[-1]
        d0, d1 = o["doc_range"]
        assert (d0, d1) == (want_bounds[r], want_bounds[r + 1])
        assert o["docs"] == ref["docs"][d0:d1]
        a, b = rptr[d0], rptr[d1]
        assert o["ptr"] == (rptr[d0:d1 + 1] - a).tolist()
        assert o["widx"] == ref["widx"][a:b] and o["cnt"] == ref["cnt"][a:b]


def test_byte_ranges_partition_lines(tmp_path):
    from oni_ml_amd.features.flow_dist import byte_ranges
    from oni_ml_amd.ops import native
    paths = []
    for i in range(3):
        p = tmp_path / f"f{i}.csv"
        p.write_text("a,b\n" + "".join(f"{i * 1000 + j},x\n" for j in range(97 + 13 * i)))
        paths.append(str(p))
    want = [int(l.split(",")[0]) for p in paths for l in open(p).read().splitlines()[1:]]
    for world in (1, 2, 5, 16):
        got = []
        for r in range(world):
            t = native.lib().TextTable(2, [0], [[1]])
            for p, b, e in byte_ranges(paths, world, r):
                t.load_range(p, b, e, "a,b", True, 1)
            got += t.numeric(0).astype(int).tolist()
        assert got == want, world
