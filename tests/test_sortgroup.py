"""ops/sortgroup.py against the torch ops it stands in for (torch.unique / sort / repeat_interleave / diff /
boolean-mask compaction), bit for bit, on the CPU and (gpu marker) on the device."""
import numpy as np
import pytest
import torch

from oni_ml_amd.ops import sortgroup as SG


def _f64_cases(rng):
    base = rng.integers(-50, 50, 4000).astype(np.float64) * 0.25
    extra = np.array([np.inf, -np.inf, 1e308, -1e308, 5e-324, -5e-324, 0.0, 1.0, -1.0])
    x = np.concatenate([base, extra, base[:100]])
    rng.shuffle(x)
    return x


def _same(a, b):
    a, b = a.cpu(), b.cpu()
    assert a.dtype == b.dtype and a.shape == b.shape
    if a.dtype == torch.float64:
        assert np.array_equal(a.numpy().view(np.int64), b.numpy().view(np.int64))
    else:
        assert torch.equal(a, b)


def _check_all(dev):
    rng = np.random.default_rng(0)
    x = torch.from_numpy(_f64_cases(rng)).to(dev)
    # float64 order keys: the stable sort equals torch's (no -0.0 / NaN ties in these values)
    sv, sp = SG.sort_stable(x)
    rv, rp = torch.sort(x, stable=True)
    _same(sv, rv)
    _same(sp, rp)
    for t in (x, torch.from_numpy(rng.integers(-(1 << 40), 1 << 40, 5000)).to(dev),
              torch.from_numpy(rng.integers(0, 30, 5000)).to(dev)):
        u, inv, cnt = SG.unique(t, return_inverse=True, return_counts=True)
        ru, rinv, rcnt = torch.unique(t, sorted=True, return_inverse=True, return_counts=True)
        _same(u, ru)
        _same(inv, rinv)
        _same(cnt, rcnt.to(torch.int64))
        _same(SG.unique(t), ru)
        w = torch.from_numpy(rng.integers(1, 1000, t.numel())).to(dev)
        k, s = SG.segment_sums(t, w)
        rs = torch.zeros(ru.numel(), dtype=torch.int64, device=dev).index_add_(0, rinv, w)
        _same(k, ru)
        _same(s, rs)
    lens = torch.from_numpy(rng.integers(0, 6, 300)).to(dev)
    _same(SG.segment_ids(lens), torch.repeat_interleave(torch.arange(300, device=dev), lens))
    _same(SG.segment_ids(lens, int(lens.sum())), torch.repeat_interleave(torch.arange(300, device=dev), lens))
    v = torch.from_numpy(rng.integers(0, 100, 50)).to(dev)
    _same(SG.diff_prepend0(v), torch.diff(v, prepend=v.new_zeros(1)))
    keep = torch.from_numpy(rng.random(5000) < 0.3).to(dev)
    vals = torch.from_numpy(rng.integers(0, 1 << 30, 5000).astype(np.int32)).to(dev)
    c, before = SG.compact(vals, keep)
    _same(c, vals[keep])
    _same(before[1:], torch.cumsum(keep.to(torch.int64), 0))
    # empty inputs
    e = torch.zeros(0, dtype=torch.int64, device=dev)
    assert SG.unique(e).numel() == 0
    assert SG.segment_ids(e).numel() == 0
    assert SG.compact(e, e.to(torch.bool))[0].numel() == 0


def test_sortgroup_matches_torch_cpu():
    _check_all(torch.device("cpu"))


def test_f64_keys_zero_and_nan_order():
    """-0.0 sorts just below +0.0 (one unique group under !=, the first of the run kept: -0.0); NaN of
    either sign last and never merged, as torch.unique's adjacent test leaves them."""
    nan_neg = np.frombuffer(np.array([0xFFF8000000000000], np.uint64).tobytes(), np.float64)[0]
    x = torch.tensor([0.0, np.nan, -0.0, 2.0, nan_neg, -3.0, 0.0], dtype=torch.float64)
    sv, _ = SG.sort_stable(x)
    assert sv[:4].tolist()[0] == -3.0 and np.signbit(sv[1].item()) and not np.signbit(sv[2].item())
    assert np.isnan(sv[-1].item()) and np.isnan(sv[-2].item())
    u = SG.unique(x)
    assert u.numel() == 5 and np.signbit(u[1].item()) and u[2].item() == 2.0


@pytest.mark.gpu
def test_sortgroup_matches_torch_gpu():
    _check_all(torch.device("cuda"))
