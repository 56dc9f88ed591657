"""The sharded pipeline's non-replicating collectives (parallel/shardio.py) at 3 ranks over gloo, against
their one-process definitions: the hash-partitioned first-appearance dictionary, row fetches from
row-range shards, range slices built from (id, row) pairs and the hash-partitioned name map."""
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_dist import _free_port  # noqa: E402


def _names(rank):
    rng = np.random.default_rng(rank)
    pool = [f"10.{i // 256}.{i % 256}.1" for i in range(300)] + ["", "x\x00", "x", "a" * 37]
    # each rank's local dictionary: distinct names in local first-appearance order
    seq = [pool[i] for i in rng.integers(0, len(pool), 400)]
    return list(dict.fromkeys(seq))


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(1)
    try:
        from oni_ml_amd.parallel import dist as D
        from oni_ml_amd.parallel import shardio as S
        ctx = D.init_from_env(backend="gloo")
        names = _names(rank)
        data, off = S.names_to_bytes(names)
        tab, lmap = S.first_appearance(ctx, data, off)
        got_names = tab.take(lmap)
        # fetch_rows: a [D, 3] table split in uneven row ranges; any order, repeats and -1
        D_ = 50
        starts = [0, 7, 7, D_]
        full = np.arange(D_ * 3, dtype=np.float64).reshape(D_, 3)
        local = full[starts[rank]:starts[rank + 1]]
        rng = np.random.default_rng(10 + rank)
        qry = rng.integers(-1, D_, 40)
        rows = S.fetch_rows(ctx, local, starts, qry)
        # range_put: every rank sends the (id, value) pairs of its own ids
        total = 31
        ids = np.arange(rank, total, world)
        sl = S.range_put(ctx, ids, ids * 10, total, fill=-1)
        # DistDict: later (larger) values win for repeated names
        dd = S.DistDict(ctx, [f"w{(i * 7 + rank) % 23}" for i in range(10)], np.arange(10) + 100 * rank)
        look = dd.lookup([f"w{i}" for i in range(25)] + ["z" * 50])
        q.put((rank, dict(names=names, lmap=lmap.tolist(), got=got_names, total=len(tab), qry=qry.tolist(),
                          rows=rows.tolist(), slice=sl.tolist(), look=look.tolist())))
        ctx.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


def test_shardio_collectives_match_one_process():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in range(world):
        assert isinstance(out[r], dict), out[r]
    # first appearance over the concatenation in rank order
    concat = [n for r in range(world) for n in out[r]["names"]]
    want = list(dict.fromkeys(concat))
    gid = {n: i for i, n in enumerate(want)}
    for r in range(world):
        o = out[r]
        assert o["total"] == len(want)
        assert o["lmap"] == [gid[n] for n in o["names"]]
        assert o["got"] == o["names"]                      # names come back exactly (NUL and empty kept)
    full = np.arange(50 * 3, dtype=np.float64).reshape(50, 3)
    for r in range(world):
        qry = np.asarray(out[r]["qry"])
        exp = np.where((qry >= 0)[:, None], full[np.maximum(qry, 0)], 0.0)
        assert np.array_equal(np.asarray(out[r]["rows"]), exp)
    sl = np.concatenate([out[r]["slice"] for r in range(world)])
    assert np.array_equal(sl, np.arange(31) * 10)
    # DistDict: name -> max value over every rank's entries
    best = {}
    for r in range(world):
        for i in range(10):
            k = f"w{(i * 7 + r) % 23}"
            best[k] = max(best.get(k, -1), i + 100 * r)
    exp = [best.get(f"w{i}", -1) for i in range(25)] + [-1]
    for r in range(world):
        assert out[r]["look"] == exp
