"""Fail-fast stage runner with completion markers, timing and a run lock.

The reference chains stages in bash with no exit-code checks (ml_ops.sh has no
`set -e`), fixed `sleep`s as synchronisation and bare `time` prefixes
(ml_ops.sh:57,67,80,84,108).  Here:

* every stage is timed (roctx range + metrics.jsonl record with wall seconds);
* an exception stops the run immediately and is recorded (non-zero exit);
* a finished stage writes ``<LPATH>/.stages/<name>.done`` (JSON with its
  outputs); with ``resume=True`` finished stages are skipped and the run
  restarts at the first incomplete one;
* ``<LPATH>/.lock`` (O_EXCL) stops two runs for the same day from clobbering
  the working directory (the reference's implicit hazard).
"""
from __future__ import annotations

import json
import os
import time
import traceback
from contextlib import contextmanager
from typing import Optional

from ..utils.trace import range_pop, range_push


class StageFailed(RuntimeError):
    pass


class RunLock:
    def __init__(self, path: str):
        self.path = path
        self.fd = None

    def __enter__(self):
        try:
            self.fd = os.open(self.path, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644)
        except FileExistsError:
            pid = ""
            try:
                pid = open(self.path).read().strip()
            except OSError:
                pass
            if pid.isdigit() and not _alive(int(pid)):
                os.unlink(self.path)   # stale lock of a dead run
                self.fd = os.open(self.path, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644)
            else:
                raise RuntimeError(f"another run holds {self.path} (pid {pid or '?'})")
        os.write(self.fd, str(os.getpid()).encode())
        return self

    def __exit__(self, *exc):
        if self.fd is not None:
            os.close(self.fd)
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


class StageRunner:
    def __init__(self, workdir: str, resume: bool = False, rank: int = 0, metrics_name: str = "metrics.jsonl",
                 log=print, sync=None):
        self.workdir = workdir
        self.resume = resume
        self.rank = rank
        self.mdir = os.path.join(workdir, ".stages")
        # rank 0: metrics.jsonl; rank r > 0: metrics.rank<r>.jsonl (per-rank stage times of a sharded run)
        base, ext = os.path.splitext(metrics_name)
        self.metrics = os.path.join(workdir, metrics_name if rank == 0 else f"{base}.rank{rank}{ext}")
        self.log = log
        self.sync = sync
        self.times = {}
        self._pending = []          # (name, record, join): stages whose outputs are still being written
        if rank == 0:
            os.makedirs(self.mdir, exist_ok=True)

    def done(self, name: str) -> bool:
        return self.resume and os.path.exists(os.path.join(self.mdir, name + ".done"))

    def info(self, name: str) -> dict:
        p = os.path.join(self.mdir, name + ".done")
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f)
        return {}

    def clear(self):
        if self.rank == 0 and os.path.isdir(self.mdir):
            for f in os.listdir(self.mdir):
                os.unlink(os.path.join(self.mdir, f))

    def emit(self, rec: dict):
        with open(self.metrics, "a") as f:
            f.write(json.dumps(dict(rec, rank=self.rank)) + "\n")

    @contextmanager
    def stage(self, name: str, **meta):
        """Run a stage body; record time; write the completion marker with `result` dict entries."""
        result = {}
        range_push(name)
        if self.sync:
            self.sync()
        t0 = time.perf_counter()
        try:
            yield result
            if self.sync:
                self.sync()
        except Exception as e:
            dt = time.perf_counter() - t0
            self.emit(dict(stage=name, status="failed", seconds=dt, error=repr(e), ts=time.time()))
            if self.rank == 0:
                self.log(f"[stage {name}] FAILED after {dt:.3f}s: {e!r}")
                self.log(traceback.format_exc())
            raise
        finally:
            range_pop()
        dt = time.perf_counter() - t0
        self.times[name] = self.times.get(name, 0.0) + dt
        join = result.pop("_defer", None)
        rec = dict(stage=name, status="ok", seconds=dt, ts=time.time(), **meta,
                   **{k: v for k, v in result.items() if isinstance(v, (int, float, str, bool))})
        self.emit(rec)
        if join is not None:
            # the stage's results are in memory (later stages use them now); its files are still
            # being written in the background: the completion marker waits for them (finish_deferred)
            self._pending.append((name, rec, join))
            if self.rank == 0:
                self.log(f"[stage {name}] {dt:.3f}s (files pending)")
            return
        self._mark(name, rec)
        if self.rank == 0:
            self.log(f"[stage {name}] {dt:.3f}s")

    def _mark(self, name: str, rec: dict):
        if self.rank == 0:
            with open(os.path.join(self.mdir, name + ".done"), "w") as f:
                json.dump(rec, f)

    def finish_deferred(self, suppress: bool = False):
        """Wait for background output writers; a stage is marked complete only once its files are.
        ``suppress``: another error is already propagating -- drain the writers, raise nothing.  That
        path may run on one rank only, so a join with an ``abort`` attribute (a writer whose completion
        is collective, e.g. the LDA part files' concatenation) runs ``abort`` instead: local work only,
        and no stage is marked complete."""
        pending, self._pending = self._pending, []
        err = None
        for name, rec, join in pending:
            t0 = time.perf_counter()
            if suppress and hasattr(join, "abort"):
                try:
                    join.abort()
                except Exception:  # noqa: BLE001 -- an error is already propagating
                    pass
                continue
            try:
                join()
            except Exception as e:  # noqa: BLE001 -- re-raised after the other writers finished
                self.emit(dict(stage=name, status="failed", seconds=0.0, error=repr(e), ts=time.time()))
                err = err or e
                continue
            wait = time.perf_counter() - t0
            rec = dict(rec, files_wait_seconds=wait)
            self.emit(dict(stage=name + ".files", status="ok", seconds=wait, ts=time.time()))
            self._mark(name, rec)
        if err is not None and not suppress:
            raise StageFailed(f"background writes failed: {err!r}") from err

    def skip(self, name: str):
        if self.rank == 0:
            self.log(f"[stage {name}] already complete (resume), skipped")
        self.emit(dict(stage=name, status="skipped", seconds=0.0, ts=time.time()))
