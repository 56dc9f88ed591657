"""roctx ranges + structured stage timers (SURVEY.md §5.1 tracing).

The reference only wraps five stages in bash `time` (ml_ops.sh:57,67,80,84,108).
Here every stage and every EM iteration (E-step / all-reduce / M-step) can be
bracketed with roctx ranges that show up in `rocprofv3 --marker-trace`
timelines, and a StageTimer records wall time per stage into metrics.jsonl.
roctx is enabled with ONI_ROCTX=1 (a no-op otherwise, so hot loops pay nothing).
"""
from __future__ import annotations

import ctypes
import json
import os
import time
from contextlib import contextmanager

_roctx = None
_enabled = os.environ.get("ONI_ROCTX", "0") == "1"


def _load():
    global _roctx, _enabled
    if _roctx is not None or not _enabled:
        return
    for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            return
        except OSError:
            continue
    _enabled = False


def range_push(name: str):
    if not _enabled:
        return
    _load()
    if _roctx is not None:
        _roctx.roctxRangePushA(name.encode())


def range_pop():
    if not _enabled:
        return
    if _roctx is not None:
        _roctx.roctxRangePop()


def mark(name: str):
    if _enabled:
        _load()
        if _roctx is not None:
            _roctx.roctxMarkA(name.encode())


@contextmanager
def trace_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


class StageTimer:
    """Collects {stage: seconds} and appends JSON records to a metrics file."""

    def __init__(self, metrics_path=None, rank: int = 0, sync_cuda: bool = True):
        self.records = []
        self.metrics_path = metrics_path
        self.rank = rank
        self.sync_cuda = sync_cuda

    def _sync(self):
        if self.sync_cuda:
            try:
                import torch
                if torch.cuda.is_available() and torch.cuda.is_initialized():
                    torch.cuda.synchronize()
            except Exception:
                pass

    @contextmanager
    def stage(self, name: str, **extra):
        range_push(name)
        self._sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self._sync()
            dt = time.perf_counter() - t0
            range_pop()
            rec = dict(stage=name, seconds=dt, rank=self.rank, ts=time.time(), **extra)
            self.records.append(rec)
            self.emit(rec)

    def emit(self, rec: dict):
        if self.metrics_path and self.rank == 0:
            with open(self.metrics_path, "a") as f:
                f.write(json.dumps(rec) + "\n")

    def summary(self) -> dict:
        out = {}
        for r in self.records:
            out[r["stage"]] = out.get(r["stage"], 0.0) + r["seconds"]
        return out
