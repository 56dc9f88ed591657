"""End-to-end suspicious-connects pipelines (flow / dns), the ml_ops.sh replacement."""
from __future__ import annotations


def run(cfg, dist=None, device=None, log=print) -> dict:
    cfg.validate()
    import os
    if dist is None or dist.rank == 0:
        os.makedirs(cfg.lpath, exist_ok=True)
    rank0 = dist is None or dist.rank == 0
    hd = None
    if cfg.hdfs:
        from ..io.hdfs import Hdfs
        hd = Hdfs(cfg.hadoop)
        if rank0:   # featurization and scoring run on rank 0 (ml_ops.sh:57-62 staging)
            stage = os.path.join(cfg.lpath, ".hdfs_in")
            if cfg.dsource == "flow":
                cfg.flow_path = hd.stage_inputs(cfg.flow_path, stage)
            else:
                cfg.dns_path = hd.stage_inputs(cfg.dns_path, stage)
    if cfg.dsource == "flow":
        from .flow import run as _run
    else:
        from .dns import run as _run
    summary = _run(cfg, dist=dist, device=device, log=log)
    if hd is not None and rank0:
        if not cfg.hpath:
            raise ValueError("--hdfs needs HPATH")
        hd.publish(cfg.lpath, cfg.hpath, cfg.dsource)     # ml_ops.sh:93-101,110-115
        summary["hdfs_published"] = cfg.hpath
    return summary
