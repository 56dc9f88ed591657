"""End-to-end suspicious-connects pipelines (flow / dns), the ml_ops.sh replacement."""
from __future__ import annotations


def run(cfg, dist=None, device=None, log=print) -> dict:
    cfg.validate()
    import os
    if dist is None or dist.rank == 0:
        os.makedirs(cfg.lpath, exist_ok=True)
    if cfg.dsource == "flow":
        from .flow import run as _run
    else:
        from .dns import run as _run
    return _run(cfg, dist=dist, device=device, log=log)
