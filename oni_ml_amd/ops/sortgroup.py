"""Sort-based group-by on the device from the few torch kernels a pipeline stage runs anyway (the int64 radix
sort, cumsum, searchsorted, elementwise ops, index_select / index_put).

In a fresh process the HIP runtime loads a torch source file's code object on the first call of any kernel
in it.  ``scripts/micro/first_op_cost.py`` (``profiles/r6ae_first_op_cost.md``: each op alone in a fresh
process on an MI355X) measured first calls of 120 ms for ``torch.maximum``, 80 ms for a float64 sort against
20 ms for the int64 one, 50 ms ``bincount``, 48 ms ``unique``, 46 ms advanced indexing against 4 ms
``index_select``, 36 ms ``repeat_interleave`` and 35 ms ``nonzero`` -- against < 1 ms for each call once
loaded.  A cold ``ml_ops`` process (the reference's ml_ops.sh runs every stage as a fresh process) paid them
in flow_pre, lda_pre and the engine setup.  The helpers below return what those ops return, bit for bit
(``tests/test_sortgroup.py``), from kernels the stages load anyway; they run on any device.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

_LOW63 = 0x7FFFFFFFFFFFFFFF


def gather(x: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """x[idx] for a 1-D (or row-major N-D, along dim 0) tensor and an integer index vector."""
    return x.index_select(0, idx.reshape(-1).to(torch.int64))


def f64_order_keys(x: torch.Tensor) -> torch.Tensor:
    """int64 keys whose signed order is torch.sort's order of the float64 values: IEEE bits with the low 63
    bits of negatives flipped (-0.0 just below +0.0), every NaN made the canonical positive NaN first (torch
    sorts NaN after +inf whatever its sign bit)."""
    x = torch.where(x != x, torch.full_like(x, float("nan")), x)
    k = x.contiguous().view(torch.int64)
    return torch.where(k < 0, k ^ _LOW63, k)


def sort_stable(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(sorted values, permutation) = torch.sort(x, stable=True) of a 1-D tensor; float64 through its int64
    order keys (one radix sort kernel family for every dtype the stages sort)."""
    if x.dtype == torch.float64:
        _, perm = torch.sort(f64_order_keys(x), stable=True)
        return gather(x, perm), perm
    return torch.sort(x, stable=True)


def run_ids(sk: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """Group index of every position of a sorted 1-D tensor -- runs of equal values under ``!=`` (so
    -0.0 / +0.0 share a run and NaN != NaN, as torch.unique's adjacent test) -- and the number of groups.
    One host sync (the group count)."""
    n = sk.numel()
    new = torch.ones(n, dtype=torch.int64, device=sk.device)
    if n > 1:
        new[1:] = (sk[1:] != sk[:-1]).to(torch.int64)
    grp = torch.cumsum(new, 0) - 1
    return grp, (int(grp[-1]) + 1 if n else 0)


_SPILL = 1024   # scatter targets for the positions a scatter drops (spread: one address would serialise)


def run_starts(grp: torch.Tensor, G: int) -> torch.Tensor:
    """First position of each of the G runs of a group-index vector (``run_ids``), int64 [G + 1], n last.
    One scatter over the positions (a binary search per run cost O(G log n) random reads: ~0.3 s per
    count_pairs at config 5's 100 M rows and ~40 M distinct pairs)."""
    n = grp.numel()
    pos = torch.arange(n, device=grp.device, dtype=torch.int64)
    first = torch.ones(n, dtype=torch.bool, device=grp.device)
    if n > 1:
        first[1:] = grp[1:] != grp[:-1]
    st = torch.empty(G + 1 + _SPILL, dtype=torch.int64, device=grp.device)
    st.index_put_((torch.where(first, grp, (G + 1) + (pos & (_SPILL - 1))),), pos)
    st[G] = n
    return st[:G + 1]


def unique(x: torch.Tensor, return_inverse: bool = False, return_counts: bool = False):
    """torch.unique(x, sorted=True, return_inverse, return_counts) of a 1-D tensor: the first value of every
    run of the stably sorted values; inverse and counts int64."""
    x = x.reshape(-1)
    sk, perm = sort_stable(x)
    grp, G = run_ids(sk)
    st = run_starts(grp, G)
    out = [gather(sk, st[:-1])]
    if return_inverse:
        inv = torch.empty_like(grp)
        inv[perm] = grp
        out.append(inv)
    if return_counts:
        out.append(st[1:] - st[:-1])
    return out[0] if len(out) == 1 else tuple(out)


def segment_sums(keys: torch.Tensor, w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(sorted distinct keys, sum of the integer weights w per key): a radix sort and a prefix sum, no
    atomics (heavily repeated keys cost nothing extra; an int64 index_add_ over a handful of hot keys
    serialises on their addresses)."""
    sk, perm = sort_stable(keys.reshape(-1))
    grp, G = run_ids(sk)
    st = run_starts(grp, G)
    cw = torch.cumsum(gather(w.reshape(-1).to(torch.int64), perm), 0)
    tot = gather(cw, st[1:] - 1)
    return gather(sk, st[:-1]), diff_prepend0(tot)


def segment_ids(lens: torch.Tensor, total: Optional[int] = None) -> torch.Tensor:
    """torch.repeat_interleave(arange(len(lens)), lens): the segment of every position, int64 [sum(lens)]
    (empty segments skipped, as repeat_interleave does).  ``total``: sum(lens) when known (no host sync)."""
    lens = lens.reshape(-1).to(torch.int64)
    ends = torch.cumsum(lens, 0)
    if total is None:
        total = int(ends[-1]) if lens.numel() else 0
    total = int(total)
    dev = lens.device
    # O(n): a 1 at the first position of every non-empty segment, a prefix sum numbers them, and the ids
    # of the non-empty segments map that number back (a binary search per position read O(n log D))
    nonempty = lens > 0
    ids, _ = compact(torch.arange(lens.numel(), device=dev, dtype=torch.int64), nonempty)
    starts, _ = compact(ends - lens, nonempty)
    marks = torch.zeros(total, dtype=torch.int64, device=dev)
    if ids.numel():
        marks.index_put_((starts,), torch.ones_like(starts))
    return gather(ids, torch.cumsum(marks, 0) - 1) if total else marks


def diff_prepend0(x: torch.Tensor) -> torch.Tensor:
    """torch.diff(x, prepend=zeros(1)) of a 1-D tensor."""
    out = torch.empty_like(x)
    if x.numel():
        out[:1] = x[:1]
        out[1:] = x[1:] - x[:-1]
    return out


def compact(x: torch.Tensor, keep: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(x[keep], exclusive prefix count of keep [n + 1]) for a 1-D x and a bool mask, order kept, without
    nonzero: kept elements are scattered to their prefix positions, the dropped ones to a spill slot."""
    k = keep.reshape(-1).to(torch.int64)
    csum = torch.zeros(k.numel() + 1, dtype=torch.int64, device=x.device)
    csum[1:] = torch.cumsum(k, 0)
    total = int(csum[-1])
    spill = total + (torch.arange(k.numel(), device=x.device, dtype=torch.int64) & (_SPILL - 1))
    dest = torch.where(keep.reshape(-1), csum[:-1], spill)
    out = torch.empty(total + _SPILL, dtype=x.dtype, device=x.device)
    out.index_put_((dest,), x.reshape(-1))      # dropped values land in the spill slots past total
    return out[:total], csum
