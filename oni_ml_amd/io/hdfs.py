"""Optional HDFS hooks around the local-FS pipeline (reference ml_ops.sh HDFS steps).

The reference moves data through HDFS between its Spark and local stages:

  * ``hadoop fs -copyToLocal ${HPATH}/word_counts/part-*``   (ml_ops.sh:59)   -- not needed here:
    the featurizer hands the corpus to the LDA stage in memory;
  * ``hadoop fs -rm/-put doc_results.csv, word_results.csv ${HPATH}``  (ml_ops.sh:93-96);
  * ``hadoop fs -rm -R -f ${HPATH}/word_counts ${HPATH}/scored``       (ml_ops.sh:100-101);
  * ``hadoop fs -copyToLocal ${HPATH}/scored/part-*`` -> ``${DSOURCE}_results.csv`` (ml_ops.sh:110-115).

This engine reads and writes the local FS.  With ``--hdfs``, ``hdfs://`` inputs are staged to
``LPATH/.hdfs_in`` first (``stage_inputs``) and the results are published back to ``HPATH`` in the
reference layout (``publish``): the model tables at ``HPATH/*.csv`` and the scored rows at
``HPATH/scored/part-00000``.  Every step is one ``hadoop fs`` subprocess; a missing ``hadoop``
binary is an error, never a silent skip.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from typing import Callable, List, Optional


def is_hdfs(path: str) -> bool:
    return path.startswith("hdfs://") or path.startswith("viewfs://")


class Hdfs:
    def __init__(self, hadoop: str = "hadoop", runner: Optional[Callable[[List[str]], None]] = None):
        self.hadoop = hadoop
        self._run = runner or self._subprocess

    def _subprocess(self, cmd: List[str]):
        if shutil.which(cmd[0]) is None and not os.path.exists(cmd[0]):
            raise FileNotFoundError(f"HDFS step needs the hadoop CLI ({cmd[0]!r} not found)")
        subprocess.run(cmd, check=True)

    def fs(self, *args: str, check: bool = True):
        try:
            self._run([self.hadoop, "fs", *args])
        except subprocess.CalledProcessError:
            if check:
                raise

    def stage_inputs(self, path_spec: str, local_dir: str) -> str:
        """Copy every hdfs:// entry of a comma-separated path list to local_dir; returns the local spec."""
        out = []
        for i, p in enumerate(x for x in path_spec.split(",") if x):
            if is_hdfs(p):
                dst = os.path.join(local_dir, f"in{i:03d}")
                os.makedirs(dst, exist_ok=True)
                self.fs("-copyToLocal", p.rstrip("/") + "/*" if not os.path.splitext(p)[1] else p, dst)
                out.append(dst)
            else:
                out.append(p)
        return ",".join(out)

    def publish(self, lpath: str, hpath: str, dsource: str):
        """The reference's post-LDA HDFS layout (ml_ops.sh:93-101) plus the scored rows."""
        for name in ("doc_results.csv", "word_results.csv"):
            self.fs("-rm", f"{hpath}/{name}", check=False)
            self.fs("-put", os.path.join(lpath, name), f"{hpath}/.")
        self.fs("-rm", "-R", "-f", f"{hpath}/word_counts", check=False)
        self.fs("-rm", "-R", "-f", f"{hpath}/scored", check=False)
        self.fs("-mkdir", "-p", f"{hpath}/scored")
        self.fs("-put", os.path.join(lpath, f"{dsource}_results.csv"), f"{hpath}/scored/part-00000")
