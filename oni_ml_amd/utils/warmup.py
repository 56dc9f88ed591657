"""Cold-process start-up: overlap the GPU runtime's one-time costs with work the process must do anyway.

``ml_ops`` runs as a fresh process per day (the reference times each stage as a fresh process,
ml_ops.sh:57,67,80,84,108).  A fresh process pays, before its first useful kernel: the HIP runtime and
device context, and the lazy load of every code object at its first launch (the engine's gfx950
kernels in ``_onihip``, torch's sort / unique / scan kernels).  Two overlaps:

* ``early_hip_init``: the HIP runtime + primary context of this rank's device on a thread, before
  ``import torch`` -- the ctypes call releases the GIL, so it runs while the interpreter imports torch.
  OFF by default (``ONI_EARLY_HIP=1`` enables it): with the runtime initialised from that thread
  while torch imported, the config-5 EM ran 25 iterations in 9.25-9.29 s in the five runs whose torch
  import was quick and 5.89-5.93 s in the two whose import took 11 s (the thread long finished), and
  6.00-6.09 s in all three runs without it (profiles/r4_config5.md): the E-step is 1.55x slower when
  the runtime comes up racing torch's first HIP calls.  Its start-up gain was ~0.05 s;
* ``start``: after the imports, a thread issues tiny versions of the first stages' GPU work (the torch
  ops featurization and the corpus builder use, one launch of each engine kernel family) on its own
  stream while the main thread parses the input files on the CPU.

Neither changes a result: the warm-up works on private tensors, on its own stream.

Measured (profiles/r4_cold_start.md, 3 alternating A/B pairs): the warm-up thread made the cold run
slower, not faster -- its imports and launches contend with the main thread's parsing for the GIL and
the import lock (flow_pre 0.17-0.89 s vs 0.23-0.24 s) -- so ``start`` is off unless ONI_WARMUP=1.
"""
from __future__ import annotations

import os
import threading


def early_hip_init(local_rank: int = 0):
    """Start HIP runtime + context creation for ``local_rank`` on a daemon thread (no torch needed).
    Returns the thread (or None when there is no HIP runtime)."""
    if os.environ.get("ONI_EARLY_HIP", "0") == "0":
        return None

    def run():
        try:
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
            n = ctypes.c_int(0)
            if hip.hipGetDeviceCount(ctypes.byref(n)) != 0 or n.value <= local_rank:
                return
            hip.hipSetDevice(ctypes.c_int(local_rank))
            hip.hipFree(ctypes.c_void_p(0))         # forces the primary context
        except Exception:  # noqa: BLE001 -- a missing runtime only means nothing to overlap
            pass

    t = threading.Thread(target=run, name="oni-early-hip", daemon=True)
    t.start()
    return t


def start(device):
    """Warm the first stages' GPU code on a background thread; returns the thread (or None on CPU)."""
    import torch
    device = torch.device(device)
    if device.type != "cuda" or os.environ.get("ONI_WARMUP", "0") == "0":
        return None

    def run():
        try:
            with torch.cuda.device(device):
                s = torch.cuda.Stream(device=device)
                with torch.cuda.stream(s):
                    _kernels(device)
                s.synchronize()
        except Exception:  # noqa: BLE001 -- a failed warm-up costs only the overlap
            pass

    t = threading.Thread(target=run, name="oni-warmup", daemon=True)
    t.start()
    return t


def _kernels(device):
    import numpy as np
    import torch
    from ..corpus.builder import count_pairs
    from ..ops import hip as H
    # featurization / corpus builder: radix sorts, unique, scans, searches, gathers on the dtypes they use
    n = 4096
    x = torch.arange(n, device=device, dtype=torch.int64).flip(0)
    f = x.to(torch.float64) * 0.5
    torch.sort(x, stable=True)
    torch.sort(f, stable=True)
    torch.unique(x, return_inverse=True, return_counts=True)
    torch.unique(f, return_inverse=True)
    torch.cumsum(x, 0)
    torch.searchsorted(torch.sort(f).values, f)
    torch.bincount(x % 97, minlength=97)
    torch.repeat_interleave(torch.arange(64, device=device), torch.full((64,), 2, device=device))
    count_pairs(x % 50, x % 7, torch.ones_like(x))
    # the engine's code object (one module: the first launch loads every kernel of it)
    if H.available():
        part = torch.zeros(2, 4, dtype=torch.float64, device=device)
        H.colsum_partials(part, 2, torch.zeros(4, dtype=torch.float64, device=device))
        cuts = torch.tensor([0.5, 1.5], dtype=torch.float64, device=device)
        H.bin_columns([f], [cuts])
        KS = H.padded_topics(20)
        cw = torch.ones(8, KS, dtype=torch.float64, device=device)
        H.gs_mstep(cw, cw.sum(0), torch.empty_like(cw), 20)
    np.zeros(1)
