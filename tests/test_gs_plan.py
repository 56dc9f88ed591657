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


def test_split_plan_one_batch_longest_first(monkeypatch):
    """GSSplitPlan: G = clamp(ceil(ceil(n / U) / seg_words), 2, max_seg); longest documents first into
    one co-resident batch, the rest left to the one-workgroup team; batch arrays consistent."""
    from oni_ml_amd.ops import hip as H
    monkeypatch.setattr(H, "gs_split_launch_cap", lambda KS: 20)
    lens = np.array([82418, 5000, 30000, 4200, 9100, 100, 12000], dtype=np.int64)
    order = np.argsort(-lens, kind="stable")
    cand = order[lens[order] > 4096]
    sp = H.GSSplitPlan(cand, lens, 100, 32, "cpu", seg_words=128, max_seg=16)
    # 82418 -> W 2576 -> 16 segments; 30000 -> 938 -> 8 does not fit (16 + 8 > 20); 12000 -> 375 -> 3;
    # 9100 -> 285 -> 3 does not fit (19 + 3); 5000 -> 157 -> 2 does not fit
    assert sp.segments == {0: 16, 6: 3}
    assert sorted(sp.leftover) == [1, 2, 3, 4]      # 4200 -> 132 -> 2 does not fit either
    assert len(sp.batches) == 1
    b = sp.batches[0]
    assert b["n_blocks"] == 19 and b["docs"] == 2
    assert b["seg_doc"].tolist() == [0] * 16 + [6] * 3
    assert b["seg_index"].tolist() == list(range(16)) + [0, 1, 2]
    assert b["seg_base"].tolist() == [0] * 16 + [16] * 3
    assert b["xchg"].numel() == 2 * 19 * 2 * 101
    # several batches when allowed
    sp2 = H.GSSplitPlan(cand, lens, 100, 32, "cpu", seg_words=128, max_seg=16, max_batches=8)
    assert sp2.leftover == [] and len(sp2.batches) >= 2
    assert all(bb["n_blocks"] <= 20 for bb in sp2.batches)


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
