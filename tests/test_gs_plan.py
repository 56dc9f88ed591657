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
