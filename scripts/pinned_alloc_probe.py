#!/usr/bin/env python
"""First-use cost of pinned host buffers in a fresh process (the LAG saves' deferred copies allocate
them: log beta [K, V], gamma [D, K], class_word [V, KS] of the headline corpus).

  python scripts/pinned_alloc_probe.py
"""
import json
import time

import torch


def main():
    torch.zeros(1, device="cuda")
    torch.cuda.synchronize()
    out = []
    shapes = [(20, 63707), (124451, 20), (63707, 20), (20,)] * 3 + [(124451, 20)] * 3
    keep = []
    for s in shapes:
        t0 = time.perf_counter()
        x = torch.empty(s, dtype=torch.float64, pin_memory=True)
        dt = time.perf_counter() - t0
        keep.append(x)
        out.append(dict(shape=list(s), mb=round(x.numel() * 8 / 1e6, 2), ms=round(dt * 1e3, 3)))
    # freed and taken again: the caching host allocator's reuse
    del keep
    t0 = time.perf_counter()
    y = torch.empty((124451, 20), dtype=torch.float64, pin_memory=True)
    out.append(dict(shape=[124451, 20], reuse=True, ms=round((time.perf_counter() - t0) * 1e3, 3)))
    # a device-to-host copy into it, timed (the bytes' transfer rate)
    d = torch.randn((124451, 20), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    y.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    out.append(dict(copy_mb=round(d.numel() * 8 / 1e6, 2), ms=round((time.perf_counter() - t0) * 1e3, 3)))
    t0 = time.perf_counter()
    z = d.cpu()
    out.append(dict(pageable_copy_mb=round(d.numel() * 8 / 1e6, 2), ms=round((time.perf_counter() - t0) * 1e3, 3)))
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
