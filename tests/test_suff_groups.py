"""Per-stream suff-stats plan (ops/hip.py suff_group_plan + csc_compact, used by LDAEngine._build_suff_groups at
KS > 32), checked on the host: the direct rows, the scratch rows of shared words and the combine CSC together
give every word's class_word row exactly once, equal to the single CSC pass up to summation order.  The device
passes themselves: tests/test_gs64.py::test_suff_split_matches_single_pass (GPU)."""
import numpy as np
import torch

from oni_ml_amd.ops import hip as H


def _csc(rng, D, V, nnz_per_doc=6):
    rows = []
    for d in range(D):
        ws = rng.choice(V - 3, size=rng.integers(1, nnz_per_doc + 1), replace=False)   # words V-3.. never used
        rows += [(d, int(w)) for w in ws]
    ent = np.arange(len(rows))
    doc = np.asarray([r[0] for r in rows])
    word = np.asarray([r[1] for r in rows])
    o = np.lexsort((doc, word))                    # CSC: by word, then document
    cnt = np.bincount(word, minlength=V)
    wp = np.zeros(V + 1, np.int64)
    wp[1:] = np.cumsum(cnt)
    return wp, ent[o], doc[o], len(rows)


def _sum_rows(cphi, wp, ce, words):
    out = {}
    for w in words:
        acc = np.zeros(cphi.shape[1])
        for e in ce[wp[w]:wp[w + 1]]:
            acc = acc + cphi[e]
        out[int(w)] = acc
    return out


def test_group_plan_covers_every_word_once():
    rng = np.random.default_rng(0)
    D, V, KS = 60, 40, 3
    wp, ce, cd, nnz = _csc(rng, D, V)
    cphi = rng.random((nnz, KS))
    stream_of_doc = rng.integers(0, 3, size=D)
    wpt, cet, cdt = (torch.from_numpy(x.astype(np.int32)) for x in (wp, ce, cd))
    groups, lens = [], []
    for g in range(3):
        mask = torch.from_numpy(stream_of_doc == g)
        gwp, gce, ln = H.csc_subset(wpt, cet, cdt, mask)
        groups.append((gwp, gce))
        lens.append(ln.astype(np.int64))
    plan = H.suff_group_plan(lens, V)
    assert plan is not None
    # every word exactly once: a direct row of one stream or a shared (combined) word
    seen = np.concatenate(plan["unique"] + [plan["shared"]])
    assert np.array_equal(np.sort(seen), np.arange(V))
    assert plan["rows"] == sum(m.size for m in plan["multi"])
    cw = {}
    xs = np.zeros((plan["rows"], KS))
    for g, (gwp, gce) in enumerate(groups):
        gwp_n, gce_n = gwp.numpy().astype(np.int64), gce.numpy()
        cw.update(_sum_rows(cphi, gwp_n, gce_n, plan["unique"][g]))
        mw = plan["multi"][g]
        if mw.size:
            cwp, cce = H.csc_compact(gwp, gce, mw)
            part = _sum_rows(cphi, cwp.numpy().astype(np.int64), cce.numpy(), range(mw.size))
            for i in range(mw.size):
                xs[plan["off"][g] + i] = part[i]
    comb = _sum_rows(xs, plan["wp"], plan["ce"], plan["shared"])
    assert not set(comb) & set(cw)
    cw.update(comb)
    ref = _sum_rows(cphi, wp, ce, range(V))
    for w in range(V):
        np.testing.assert_allclose(cw[w], ref[w], rtol=1e-13, atol=0)
    # the combine lists a shared word's scratch rows in stream order
    for w in plan["shared"][:5]:
        r = plan["ce"][plan["wp"][w]:plan["wp"][w + 1]]
        owners = [next(g for g in range(3) if plan["off"][g] <= x < plan["off"][g] + plan["multi"][g].size) for x in r]
        assert owners == sorted(owners) and len(owners) >= 2


def test_group_plan_none_without_shared_words():
    lens = [np.array([2, 0, 1, 0]), np.array([0, 3, 0, 0])]
    assert H.suff_group_plan(lens, 4) is None


def test_stream_slots_late_bucket_alone():
    """LDAEngine._stream_slots (the bucket -> stream map shared by _launch_buckets and the per-stream
    suff-stats plan): at KS > 32 the 8-wave team alone on stream 1, the others round-robin over the
    remaining side streams, then the current stream (0)."""
    from types import SimpleNamespace
    from oni_ml_amd.models.lda.em import LDAEngine
    plan = [(H.GS_TEAM8, None), (H.GS_TEAM4, None), (H.GS_SMALL, None), (H.GS_TINY, None)]
    gp = SimpleNamespace(KS=104, plan=plan, split=object())       # work = [split, team8, team4, small, tiny]
    eng = SimpleNamespace(_streams=[None] * 3, _late_key=LDAEngine._late_key)
    slots = LDAEngine._stream_slots(eng, gp, late=True)
    assert slots == [2, 1, 3, 0, 2]
    assert slots.count(1) == 1
    # no late bucket: plain round-robin over the side streams, then the current one
    assert LDAEngine._stream_slots(eng, gp, late=False) == [1, 2, 3, 0, 1]
    # five streams (LDAEngine(streams=5)): four side streams
    eng5 = SimpleNamespace(_streams=[None] * 4, _late_key=LDAEngine._late_key)
    assert LDAEngine._stream_slots(eng5, gp, late=True) == [2, 1, 3, 4, 0]
