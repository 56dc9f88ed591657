"""The LAG saves' pinned-buffer pool (models/lda/em.py PinnedPool): a buffer returns to the pool when its
array and every view of it are gone, and only then is handed out again."""
import gc
import threading

import numpy as np
import torch

from oni_ml_amd.models.lda.em import PinnedPool


def _pool():
    return PinnedPool(alloc=lambda shape, dtype: torch.empty(shape, dtype=dtype))


def test_released_buffer_is_reused():
    p = _pool()
    t1, a1 = p.take((4, 5), torch.float64)
    ptr = a1.__array_interface__["data"][0]
    del t1, a1
    gc.collect()
    _, a2 = p.take((4, 5), torch.float64)
    assert a2.__array_interface__["data"][0] == ptr
    assert p.allocated == 1


def test_live_view_keeps_buffer_out_of_the_pool():
    p = _pool()
    t1, a1 = p.take((3,), torch.float64)
    view = a1[1:]
    del t1, a1
    gc.collect()
    _, a2 = p.take((3,), torch.float64)          # the first buffer is still referenced through `view`
    assert p.allocated == 2
    assert not np.shares_memory(view, a2)


def test_shapes_and_dtypes_do_not_mix():
    p = _pool()
    _, a = p.take((2, 2), torch.float64)
    del _, a
    gc.collect()
    p.take((2, 2), torch.float32)
    p.take((4,), torch.float64)
    assert p.allocated == 3


def test_release_from_another_thread():
    p = _pool()
    box = {}
    t, box["a"] = p.take((8,), torch.float64)
    del t

    def writer():
        box.pop("a").sum()                          # the writer's last use, then the array is dropped

    th = threading.Thread(target=writer)
    th.start()
    th.join()
    gc.collect()
    p.take((8,), torch.float64)
    assert p.allocated == 1
