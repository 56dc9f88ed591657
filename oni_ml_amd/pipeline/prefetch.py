"""Input prefetch while the process starts.

A cold `ml_ops` process spends ~0.7 s importing torch (libtorch's dlopen and static initialisers)
before any stage runs, and the first stage only reads the day's inputs: the 27-column flow CSV into
the native table, or the DNS parquet through Arrow -- neither needs torch, and both do their work
with the GIL released.  `cli.cmd_ml_ops` therefore starts that read on a thread before it imports
torch (single-process runs, fresh work directory), and the load stage takes the result if it was
started for the same inputs; otherwise, or if the prefetch failed, the stage reads the inputs itself
(so an input error is raised and recorded inside the stage, as before).  ``ONI_PREFETCH=0`` turns it
off.  Imports nothing heavy: this module is loaded before torch.
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, Optional, Tuple

_JOBS: Dict[tuple, Tuple[threading.Thread, dict]] = {}


def flow_key(cfg) -> tuple:
    return ("flow", cfg.flow_path, cfg.feedback_path(), cfg.dupfactor, cfg.threads)


def dns_key(cfg) -> tuple:
    return ("dns", cfg.dns_path, cfg.feedback_path(), cfg.dupfactor, cfg.strict, cfg.top1m)


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
    _JOBS.clear()
    if job is None:
        return None
    t, box = job
    t.join()
    return box.get("value")


def load_dns_inputs(dns_path, feedback_path, dupfactor, strict, top1m):
    from ..features import dns_io
    return dns_io.load_dns(dns_path, feedback_path, dupfactor, strict=strict), dns_io.load_top_domains(top1m)


def start_for(cfg) -> None:
    """Start the read of ``cfg``'s inputs (flow or dns)."""
    if cfg.dsource == "flow":
        from ..features import flow_io
        start(flow_key(cfg), flow_io.load_flow, cfg.flow_path, cfg.feedback_path(), cfg.dupfactor, cfg.threads)
    elif cfg.dsource == "dns":
        start(dns_key(cfg), load_dns_inputs, cfg.dns_path, cfg.feedback_path(), cfg.dupfactor, cfg.strict,
              cfg.top1m)
