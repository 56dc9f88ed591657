"""Host-side planning of the fp64 E-step launches (no GPU needed)."""
import numpy as np

from oni_ml_amd.ops.hip import GSPlan


def test_isolate_longest_gives_each_head_document_its_own_xcd():
    o = np.arange(100, 120, dtype=np.int32)
    for m in (1, 2, 3):
        out = GSPlan.isolate_longest(o, m)
        # every document exactly once, in order, plus empty slots
        assert out[out >= 0].tolist() == o.tolist()
        for b, d in enumerate(out):
            if b % 8 < m:
                # XCD slots of the head: the i-th head document in its first round, then empty
                assert d == (o[b] if b < m else -1)
        assert out[-1] >= 0


def test_isolate_longest_short_lists():
    assert GSPlan.isolate_longest(np.array([5, 6, 7], dtype=np.int32), 1).tolist() == [5, 6, 7]
    assert GSPlan.isolate_longest(np.array([5], dtype=np.int32), 2).tolist() == [5]


def test_split_plan_water_fills_the_longest_chain(monkeypatch):
    """GSSplitPlan: segments go to the document with the longest modelled chunk (split_chain_cycles) until the
    cap is spent or that document is at its most useful G = ceil(W / seg_words); the rest stay with the
    one-workgroup team; batch arrays consistent; the exchange buffer holds the partials and the totals rows."""
    from oni_ml_amd.ops import hip as H
    monkeypatch.setattr(H, "gs_split_launch_cap", lambda KS: 20)
    lens = np.array([82418, 5000, 30000, 4200, 9100, 100, 12000], dtype=np.int64)
    order = np.argsort(-lens, kind="stable")
    cand = order[lens[order] > 4096]
    U, KS = 32, 100
    sp = H.GSSplitPlan(cand, lens, KS, U, "cpu", max_seg=16)
    assert len(sp.batches) == 1 and not sp.fixed
    b = sp.batches[0]
    assert b["n_blocks"] == sum(sp.segments.values()) <= 20
    sw = H.split_seg_words(KS)
    gmax = {int(d): max(2, min(16, -(-(-(-int(lens[d]) // U)) // sw))) for d in cand}
    assert all(2 <= g <= gmax[d] for d, g in sp.segments.items())
    assert sp.segments[0] == max(sp.segments.values())            # the longest document the most
    assert sorted(sp.leftover + list(sp.segments)) == sorted(cand.tolist())
    t = {int(d): H.split_chain_cycles(int(lens[d]), U, sp.segments.get(int(d), 1), KS) for d in cand}
    top = max(t, key=t.get)
    # the longest modelled chain cannot shorten: at its useful maximum, or no room for its next segment
    g = sp.segments.get(top, 1)
    free = 20 - b["n_blocks"]
    assert not any(x - (g if g > 1 else 0) <= free and H.split_chain_cycles(int(lens[top]), U, x, KS) < t[top]
                   for x in range(max(2, g + 1), gmax[top] + 1))
    base = 0
    for j, (d, g) in enumerate(sp.segments.items()):
        sl = slice(base, base + g)
        assert b["seg_doc"][sl].tolist() == [d] * g and b["seg_index"][sl].tolist() == list(range(g))
        assert b["seg_base"][sl].tolist() == [base] * g and b["doc_slot"][sl].tolist() == [j] * g
        base += g
    assert b["xchg"].numel() == 2 * (b["n_blocks"] + b["docs"]) * 2 * (KS + 1)
    assert b["tab"] is None and b["tab_rows"] == 0
    # past 16 segments (the two-phase exchange) and past the LDS chunk tables: a scratch per workgroup of
    # the batch's largest chunk count
    monkeypatch.setattr(H, "gs_split_launch_cap", lambda KS: 192)
    big = np.array([443426, 54924, 30000, 9000], dtype=np.int64)
    sp = H.GSSplitPlan(np.arange(4), big, KS, 32, "cpu")
    assert sp.segments[0] == -(-(-(-443426 // 32)) // H.split_seg_words(KS)) > 100
    assert sum(sp.segments.values()) <= 192 and sp.segments.get(1, 1) >= 2
    sp = H.GSSplitPlan(np.arange(2), big, KS, 1024, "cpu")
    (b,) = sp.batches
    assert b["tab_rows"] == max(-(-n // -(-n // 1024)) for n in big[:2]) and \
        b["tab"].numel() == b["n_blocks"] * b["tab_rows"] * 2 * KS
    # several batches when allowed: the rest of the candidates in later batches
    monkeypatch.setattr(H, "gs_split_launch_cap", lambda KS: 9)
    sp2 = H.GSSplitPlan(cand, lens, KS, U, "cpu", seg_words=128, max_seg=3, max_batches=8)
    assert all(bb["n_blocks"] <= 9 for bb in sp2.batches)
    assert len(sp2.batches) >= 2 and sp2.leftover == [] and set(sp2.segments) == set(cand.tolist())
    # an explicit segment size: G = clamp(ceil(W / words), 2, max_seg), longest first, while the cap allows
    monkeypatch.setattr(H, "gs_split_launch_cap", lambda KS: 20)
    sp3 = H.GSSplitPlan(cand, lens, KS, U, "cpu", seg_words=128, max_seg=16)
    assert sp3.fixed and sp3.segments == {0: 16, 6: 3} and sorted(sp3.leftover) == [1, 2, 3, 4]


def test_csc_subset_partitions_each_word_in_order():
    """csc_subset (early / late suff-stats): the two subsets partition every word's CSC slots by
    document, each keeping the original slot order."""
    import torch
    from oni_ml_amd.corpus.csr import DeviceCorpus
    from oni_ml_amd.ops.hip import csc_subset
    from oni_ml_amd.synth.corpus import planted_corpus
    c = planted_corpus(num_docs=300, num_terms=120, num_topics=4, seed=2)
    dc = DeviceCorpus.build(c, "cpu")
    late = torch.zeros(c.num_docs, dtype=torch.bool)
    late[torch.tensor([0, 5, 17, 100, 299])] = True
    pe, ee, le = csc_subset(dc.word_ptr, dc.csc_ent, dc.csc_doc, ~late)
    pl, el, ll = csc_subset(dc.word_ptr, dc.csc_ent, dc.csc_doc, late)
    wp, ce, cd = dc.word_ptr.tolist(), dc.csc_ent.tolist(), dc.csc_doc.tolist()
    assert int(pe[-1]) + int(pl[-1]) == len(ce) and (le + ll).tolist() == np.diff(wp).tolist()
    for w in range(c.num_terms):
        slots = range(wp[w], wp[w + 1])
        assert ee[int(pe[w]):int(pe[w + 1])].tolist() == [ce[s] for s in slots if not late[cd[s]]]
        assert el[int(pl[w]):int(pl[w + 1])].tolist() == [ce[s] for s in slots if late[cd[s]]]


def test_stage_tiles_cover_each_document_in_order():
    """GSStage: per launch item, the document's positions in 64-word tiles (entry of position 0, valid
    count), the item's offset at its first tile; placement gaps (-1) take no tiles."""
    import torch

    from oni_ml_amd.ops.hip import GSStage
    dp = np.array([0, 130, 130, 200, 264], dtype=np.int64)       # lengths 130, 0, 70, 64
    st = GSStage(np.array([0, -1, 2, 3], np.int32), dp, 20, torch.device("cpu"))
    per = 10 * 64
    assert st.n_tiles == 3 + 2 + 1
    assert st.tile_ent.tolist() == [0, 64, 128, 130, 194, 200]
    assert st.tile_cnt.tolist() == [64, 64, 2, 64, 6, 64]
    assert st.stage_off.tolist() == [0, 0, 3 * per, 5 * per]
    assert st.buf.numel() == 6 * per * 2 and st.nbytes == 6 * per * 16


def test_argsort_desc_stable_matches_numpy():
    from oni_ml_amd.ops.hip import argsort_desc_stable
    rng = np.random.default_rng(2)
    for hi in (5, 300, 65535, 65536, 82418, 3_000_000):
        k = rng.integers(0, hi + 1, 20000)
        k[:50] = hi
        assert np.array_equal(argsort_desc_stable(k), np.argsort(-k, kind="stable"))
    assert argsort_desc_stable(np.zeros(0, np.int64)).size == 0
