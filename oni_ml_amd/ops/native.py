"""Loader for the C++ host runtime module `_oninative` (CSV parser, formatters, lda-c reference)."""
from __future__ import annotations

import importlib
import os
import sys

_LIB = None
_ERR = None


def lib():
    global _LIB, _ERR
    if _LIB is None:
        here = os.path.join(os.path.dirname(os.path.dirname(__file__)), "_lib")
        if here not in sys.path:
            sys.path.insert(0, here)
        try:
            _LIB = importlib.import_module("_oninative")
        except Exception as e:
            _ERR = e
            raise RuntimeError(
                f"oni_ml_amd native runtime (_oninative) is not built or failed to load: {e!r}. "
                "Run `python -m oni_ml_amd._build`.") from e
        apply_thread_budget()
    return _LIB


def apply_thread_budget() -> None:
    """The native pools' default thread count (a call that passes no ``threads``) = this rank's budget
    (knobs.threads: ONI_THREADS, else the CPUs bound to the rank within the cgroup quota); re-applied by
    utils/hostres.bind_rank once the rank is pinned."""
    if _LIB is None or not hasattr(_LIB, "set_default_threads"):
        return
    from .. import knobs
    n = int(knobs.threads(16))
    _LIB.set_default_threads(n, False)
    if hasattr(_LIB, "set_background_pool"):
        _LIB.set_background_pool(max(1, n - WRITER_RESERVE))   # every background writer's threads, together


# CPUs a background writer leaves to the rank's other threads (the one driving the GPU, the HIP runtime's):
# a writer that takes the whole cgroup quota throttles the GPU-driving thread with it
WRITER_RESERVE = 2


def background_thread_budget(share: int = 1) -> None:
    """Called on a background writer thread: marks it as one (its native calls then draw their worker
    threads from the process-wide background pool of budget - WRITER_RESERVE tokens, shared by every
    writer running at the time) and asks for at most (budget - WRITER_RESERVE) / ``share`` of them."""
    if _LIB is None:
        lib()
    from .. import knobs
    _LIB.set_default_threads(max(1, (int(knobs.threads(16)) - WRITER_RESERVE) // max(1, share)), True)


def available() -> bool:
    try:
        lib()
        return True
    except RuntimeError:
        return False
