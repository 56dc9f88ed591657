"""Input prefetch while the process starts.

A cold `ml_ops` process spends ~0.7 s importing torch (libtorch's dlopen and static initialisers)
before any stage runs, and the first stage only reads the day's inputs: the 27-column flow CSV into
the native table, or the DNS parquet through Arrow (plus dns_pre's torch-free name features) -- none of
it needs torch.  `cli.cmd_ml_ops` therefore starts that work before it imports torch (single-process
runs, fresh work directory): the flow read on a thread (native, GIL released), the DNS read in a forked
child (below), and the load stage takes the result if it was started for the same inputs; otherwise,
or if the prefetch failed, the stage reads the inputs itself (so an input error is raised and
recorded inside the stage, as before).  ``ONI_PREFETCH=0`` turns it off.  Imports nothing heavy: this
module is loaded before torch.
"""
from __future__ import annotations

import os
import threading
from typing import Callable, Dict, Optional, Tuple

_JOBS: Dict[tuple, Tuple[threading.Thread, dict]] = {}
# set by cli once `import torch` is done: host work beside the import slows it (its page faults and
# allocations contend with the import's; the flow cuts beside it cost the import ~0.1 s, r6am), so the
# flow cuts wait for it and overlap the HIP runtime's start instead
_IMPORTED = threading.Event()


def imported() -> None:
    _IMPORTED.set()


def flow_key(cfg) -> tuple:
    return ("flow", cfg.flow_path, cfg.feedback_path(), cfg.dupfactor, cfg.threads)


def dns_key(cfg) -> tuple:
    return ("dns", cfg.dns_path, cfg.feedback_path(), cfg.dupfactor, cfg.strict, cfg.top1m, cfg.threads)


def start(key: tuple, fn: Callable, *args) -> None:
    box: dict = {}

    def body():
        try:
            box["value"] = fn(*args)
        except BaseException as e:  # noqa: BLE001 -- the stage re-reads and raises it there
            box["err"] = e

    t = threading.Thread(target=body, name="oni-input-prefetch", daemon=True)
    t.start()
    _JOBS[key] = (t, box)


def take(key: tuple) -> Optional[object]:
    """The prefetched value for ``key`` (waits for it), or None: nothing started for these inputs, or
    the prefetch raised.  Every other prefetch is dropped (its thread finishes on its own)."""
    job = _JOBS.pop(key, None)
    drop_all()
    if job is None:
        return None
    t, box = job
    if t is None:                      # a forked prefetch (DNS): wait for the child, map its result
        return box["collect"]()
    t.join()
    return box.get("value")


def drop_all() -> None:
    """Drop every pending prefetch: a forked child is killed, reaped and its /dev/shm directory removed
    (cmd_ml_ops calls this in a ``finally``, so a run that fails before its load stage leaves no tmpfs
    files behind; also registered with atexit when a child is forked); a thread finishes on its own."""
    jobs = list(_JOBS.values())
    _JOBS.clear()
    for t, box in jobs:
        if t is None:
            box["drop"]()


def load_dns_inputs(dns_path, feedback_path, dupfactor, strict, top1m, threads=8):
    """(table, top-1m list, dns_pre's torch-free host features) -- the name parse, the two dictionary
    encodes and the ECDF cuts of dns_pre and dns_post run here too, beside the torch import (dns_pre
    0.41 s, 0.25 s of it the first three; the cuts 0.13 s on the device, first-use kernels included;
    profiles/r5_cold_start.md)."""
    from ..features import dns_io
    tab = dns_io.load_dns(dns_path, feedback_path, dupfactor, strict=strict)
    top = dns_io.load_top_domains(top1m)
    return tab, top, dns_io.host_features(tab, top, threads, cuts=True)


# ---- DNS: a forked child process -------------------------------------------------------------------
# On a thread the DNS read cost the torch import 0.3 s (1.0-1.1 s against 0.7-0.8 alone, at any thread
# count: pyarrow's own import and its Python-side glue hold the GIL and the import lock beside torch's),
# where the flow CSV ingest (native, GIL released) costs it nothing.  So the DNS prefetch runs in a child
# forked before anything but the standard library, numpy and this package is loaded (no GPU, no
# threads): it reads the parquet, computes the host features and hands them back through /dev/shm --
# the string columns as one Arrow IPC file (memory-mapped by the parent, zero copy), the per-row arrays
# as .npy files (memory-mapped), the name lists and scalars pickled (this process's own data).

def _dns_child(args, out_dir) -> None:
    import pickle
    import numpy as np
    tab, top, F = load_dns_inputs(*args)
    from ..features import dns_io
    pa, _, _ = dns_io._pa()
    names = list(tab.arrays)
    batch = pa.record_batch([tab.arrays[c] for c in names], names=names)
    with pa.OSFile(os.path.join(out_dir, "cols.arrow"), "wb") as f, pa.ipc.new_file(f, batch.schema) as w:
        w.write_batch(batch)
    arrays = dict(frame_len=tab.frame_len, unix_tstamp=tab.unix_tstamp, weight=tab.weight)
    arrays.update({"F_" + k: v for k, v in F.items() if isinstance(v, np.ndarray)})
    for k, v in arrays.items():
        np.save(os.path.join(out_dir, k + ".npy"), np.ascontiguousarray(v))
    meta = dict(n_raw=tab.n_raw, n_feedback=tab.n_feedback, dropped=tab.dropped, top=list(top),
                F_lists={k: v for k, v in F.items() if not isinstance(v, np.ndarray)}, arrays=list(arrays))
    with open(os.path.join(out_dir, "meta.pkl"), "wb") as f:
        pickle.dump(meta, f, protocol=pickle.HIGHEST_PROTOCOL)


def _dns_drop(pid, rfd, out_dir) -> None:
    """Kill and reap an uncollected child, remove its files (idempotent)."""
    import shutil
    import signal
    try:
        os.kill(pid, signal.SIGKILL)
    except OSError:
        pass
    try:
        os.waitpid(pid, 0)
    except ChildProcessError:
        pass
    try:
        os.close(rfd)
    except OSError:
        pass
    shutil.rmtree(out_dir, ignore_errors=True)


def _dns_collect(pid, rfd, out_dir):
    """The child's result as (DnsTable, top list, host features); None if it failed."""
    import pickle
    import shutil
    try:
        ok = os.read(rfd, 2) == b"OK"
        os.close(rfd)
        os.waitpid(pid, 0)
        if not ok:
            return None
        import numpy as np
        from ..features import dns_io
        pa, _, _ = dns_io._pa()
        with open(os.path.join(out_dir, "meta.pkl"), "rb") as f:
            meta = pickle.load(f)   # written by this process's own fork (_dns_child)
        src = pa.memory_map(os.path.join(out_dir, "cols.arrow"))
        batch = pa.ipc.open_file(src).get_batch(0)
        # copy-on-write mappings: writable like the arrays a read in this process returns
        arr = {k: np.load(os.path.join(out_dir, k + ".npy"), mmap_mode="c") for k in meta["arrays"]}
        tab = dns_io.DnsTable({c: batch.column(c) for c in batch.schema.names}, arr["frame_len"], arr["unix_tstamp"],
                              arr["weight"], meta["n_raw"], meta["n_feedback"], dropped=meta["dropped"])
        F = {k[2:]: v for k, v in arr.items() if k.startswith("F_")}
        F.update(meta["F_lists"])
        return tab, meta["top"], F
    finally:
        shutil.rmtree(out_dir, ignore_errors=True)   # the mappings stay valid after the unlink


_ATEXIT = []


def _start_dns_fork(key, args) -> bool:
    import atexit
    import tempfile
    if threading.active_count() > 1 or not os.path.isdir("/dev/shm"):
        return False
    out_dir = tempfile.mkdtemp(prefix="oni_prefetch_", dir="/dev/shm")
    rfd, wfd = os.pipe()
    pid = os.fork()
    if pid == 0:                       # child: no GPU, no threads; never returns
        code = b"ER"
        try:
            os.close(rfd)
            _dns_child(args, out_dir)
            code = b"OK"
        except BaseException:  # noqa: BLE001 -- the parent's load stage re-reads and raises it there
            pass
        finally:
            try:
                os.write(wfd, code)
            finally:
                os._exit(0)
    os.close(wfd)
    _JOBS[key] = (None, dict(collect=lambda: _dns_collect(pid, rfd, out_dir),
                             drop=lambda: _dns_drop(pid, rfd, out_dir)))
    if not _ATEXIT:
        _ATEXIT.append(atexit.register(drop_all))
    return True


# host cuts only for days up to this many rows: a cold start matters for a day's run; on a month (config 5,
# 100 M rows) the device ECDF over the GPU's bandwidth beats hashing 100 M values per column on the host
HOST_CUT_ROWS = 1 << 22


def load_flow_inputs(flow_path, feedback_path, dupfactor, threads=8, fixed_cuts=False, after_import=False):
    """The flow table and, unless the run has fixed cuts (CUT), flow_pre's ECDF cuts of every row and
    flow_post's of the raw rows computed on the host (features/cuts_host.py; the same bits as the device
    rule): the stages then skip the device ECDF, whose first run in a process loaded ~0.2 s of torch kernels
    (profiles/r6aj_cold_flow_pre.md).  Kept on ``FlowTable.host_cuts``."""
    from ..features import cuts_host, flow_io
    ft = flow_io.load_flow(flow_path, feedback_path, dupfactor, threads)
    if after_import:
        _IMPORTED.wait(timeout=60.0)
    if not fixed_cuts and ft.n <= HOST_CUT_ROWS:
        cut_all = cuts_host.flow_cuts_np(ft.table, ft.n)
        cut_raw = cut_all if ft.n_feedback == 0 else cuts_host.flow_cuts_np(ft.table, ft.n_raw)
        ft.host_cuts = dict(all=cut_all, raw=cut_raw)
    return ft


def start_for(cfg, fork: bool = True, after_import: bool = False) -> None:
    """Start the read of ``cfg``'s inputs (flow or dns).  ``fork=False`` (a profiler or tracer whose
    preloaded library may already hold the GPU, cli._tool_attached): the DNS read runs on a thread.
    ``after_import``: the flow cuts wait for ``imported()`` (the caller imports torch meanwhile)."""
    if cfg.dsource == "flow":
        start(flow_key(cfg), load_flow_inputs, cfg.flow_path, cfg.feedback_path(), cfg.dupfactor, cfg.threads,
              cfg.fixed_cuts() is not None, after_import)
    elif cfg.dsource == "dns":
        args = (cfg.dns_path, cfg.feedback_path(), cfg.dupfactor, cfg.strict, cfg.top1m, cfg.threads)
        if not (fork and _start_dns_fork(dns_key(cfg), args)):
            start(dns_key(cfg), load_dns_inputs, *args)
