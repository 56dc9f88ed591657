"""Typed run configuration.

The reference spreads configuration over five layers: positional CLI
(ml_ops.sh:4-6), the bash-sourced site file /etc/duxbay.conf (ml_ops.sh:36),
environment variables read by the Scala stages (System.getenv), hard-coded
constants (K=20, 20 MPI ranks, alpha 2.5, DUPFACTOR=1000, quantile grids) and
the lda-c settings.txt.  Here they collapse into one dataclass, resolved in
this order (later wins):

    defaults < duxbay.conf-style file < environment < explicit CLI flags

`parse_duxbay` understands the bash subset such site files use: comments,
``KEY=value`` / ``KEY="value"`` / ``KEY='value'``, arrays ``KEY=(a b c)``,
``export``, and ``$VAR`` / ``${VAR}`` expansion against earlier keys plus the
run variables FDATE, YR, MH, DY and DSOURCE that ml_ops.sh defines before
sourcing the file (ml_ops.sh:4-9).
"""
from __future__ import annotations

import os
import re
import shlex
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

from .models.lda.settings import LDASettings

ENV_KEYS = ("FLOW_PATH", "DNS_PATH", "HPATH", "LPATH", "LUSER", "TOL", "DUPFACTOR", "KRB_AUTH", "NODES", "UINODE",
            "RPATH", "LDAPATH", "SPK_EXEC", "SPK_EXEC_MEM", "TOP1M", "CUT")

_VAR = re.compile(r"\$\{([A-Za-z_][A-Za-z0-9_]*)\}|\$([A-Za-z_][A-Za-z0-9_]*)")


def _expand(s: str, env: Dict[str, str]) -> str:
    return _VAR.sub(lambda m: env.get(m.group(1) or m.group(2), ""), s)


def parse_duxbay(text: str, run_vars: Optional[Dict[str, str]] = None) -> Dict[str, object]:
    """Parse a duxbay.conf-like bash file into {KEY: str | list[str]}."""
    env: Dict[str, str] = dict(run_vars or {})
    out: Dict[str, object] = {}
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        if line.startswith("export "):
            line = line[len("export "):].strip()
        m = re.match(r"^([A-Za-z_][A-Za-z0-9_]*)=(.*)$", line)
        if not m:
            continue
        key, val = m.group(1), m.group(2).strip()
        if val.startswith("("):
            inner = val[1:val.rfind(")")] if ")" in val else val[1:]
            items = [_expand(x, env) for x in shlex.split(inner, comments=True)]
            out[key] = items
            env[key] = items[0] if items else ""
            continue
        try:
            toks = shlex.split(val, comments=True)
        except ValueError:
            toks = [val]
        if val.startswith("'"):
            v = toks[0] if toks else ""
        else:
            v = _expand(toks[0] if toks else "", env)
        out[key] = v
        env[key] = v
    return out


def run_vars(fdate: str, dsource: str) -> Dict[str, str]:
    return dict(FDATE=fdate, YR=fdate[0:4], MH=fdate[4:6], DY=fdate[6:8], DSOURCE=dsource)


@dataclass
class RunConfig:
    fdate: str = ""
    dsource: str = "flow"                 # flow | dns
    tol: float = 1e-20
    lpath: str = ""                       # local working dir (reference: ${LUSER}/ml/${FDATE})
    hpath: str = ""                       # HDFS dir in the reference; unused unless set (optional copy target)
    flow_path: str = ""
    dns_path: str = ""
    top1m: str = "top-1m.csv"
    dupfactor: int = 1000
    topics: int = 20
    alpha: float = 2.5
    process_count: int = 20               # reference MPI ranks; CPU backend shards
    gpus: int = 1
    backend: str = "auto"                 # hip | torch | cpu | auto
    compat: str = "strict"                # strict | fixed
    seed: int = 0
    start: str = "random"                 # random | seeded | <model prefix>
    resume: bool = False
    threads: int = 0      # host threads of the stage pools; 0: knobs.threads(8), this rank's CPU budget
    write_doc_wc: bool = True
    word_assignments: bool = True          # lda-c writes word-assignments.dat on every `lda est`
    rank_gamma: Optional[bool] = None      # <rank>.gamma / <rank>.beta; None: multi-rank runs of K x V <= 2^26
    verbose: bool = True
    cuts: str = ""                        # fixed flow cuts in flow_qtiles form ("ibyt,ipkt,time"; the
                                          # reference's commented-out CUT consumer, flow_pre_lda.scala:95-98)
    hdfs: bool = False                    # stage hdfs:// inputs locally and publish results to HPATH
    hadoop: str = "hadoop"                # hadoop CLI used for the HDFS steps
    settings: LDASettings = field(default_factory=LDASettings)
    extra: Dict[str, object] = field(default_factory=dict)

    def fixed_cuts(self):
        """Cuts from `cuts` (flow_qtiles text or a path to such a file), else None."""
        if not self.cuts:
            return None
        from .features.quantiles import parse_qtiles
        text = self.cuts
        if os.path.exists(text):
            with open(text) as f:
                text = f.read()
        return parse_qtiles(text)

    @property
    def strict(self) -> bool:
        return self.compat == "strict"

    def feedback_path(self) -> str:
        return os.path.join(self.lpath, f"{self.dsource}_scores.csv")

    def validate(self):
        if self.dsource not in ("flow", "dns"):
            raise ValueError("TYPE must be flow or dns")
        if self.fdate and (len(self.fdate) != 8 or not self.fdate.isdigit()):
            raise ValueError("FDATE must be YYYYMMDD")
        if self.compat not in ("strict", "fixed"):
            raise ValueError("compat must be strict or fixed")
        if not self.lpath:
            raise ValueError("LPATH (working directory) is not set")
        if self.dsource == "flow" and not self.flow_path:
            raise ValueError("FLOW_PATH is not set")
        if self.dsource == "dns" and not self.dns_path:
            raise ValueError("DNS_PATH is not set")
        if self.topics < 1:
            raise ValueError("topics must be >= 1")
        return self

    def to_dict(self) -> dict:
        d = asdict(self)
        return d


def resolve(fdate: str, dsource: str, tol: Optional[float] = None, conf_path: Optional[str] = None,
            environ: Optional[Dict[str, str]] = None, **overrides) -> RunConfig:
    """Build a RunConfig from the duxbay file, the environment and explicit overrides."""
    env = dict(os.environ if environ is None else environ)
    cfg = RunConfig(fdate=fdate, dsource=dsource)
    layers: List[Dict[str, object]] = []
    if conf_path and os.path.exists(conf_path):
        with open(conf_path) as f:
            layers.append(parse_duxbay(f.read(), run_vars(fdate, dsource)))
    layers.append({k: env[k] for k in ENV_KEYS if k in env})
    for layer in layers:
        _apply(cfg, layer)
    if tol is not None:
        cfg.tol = float(tol)
    if not cfg.lpath and isinstance(layers[0].get("LUSER") if layers else None, str):
        cfg.lpath = os.path.join(str(layers[0]["LUSER"]), "ml", fdate)
    for k, v in overrides.items():
        if v is None:
            continue
        if not hasattr(cfg, k):
            raise TypeError(f"unknown config key {k}")
        setattr(cfg, k, v)
    if cfg.threads <= 0:
        from . import knobs
        cfg.threads = knobs.threads(8)
    return cfg


def _apply(cfg: RunConfig, layer: Dict[str, object]):
    m = dict(FLOW_PATH="flow_path", DNS_PATH="dns_path", HPATH="hpath", LPATH="lpath", TOP1M="top1m")
    for k, attr in m.items():
        if k in layer and isinstance(layer[k], str) and layer[k]:
            setattr(cfg, attr, layer[k])
    if "TOL" in layer and layer["TOL"] not in ("", None):
        cfg.tol = float(layer["TOL"])
    if "DUPFACTOR" in layer and layer["DUPFACTOR"] not in ("", None):
        cfg.dupfactor = int(layer["DUPFACTOR"])
    if "CUT" in layer and isinstance(layer["CUT"], str) and layer["CUT"].strip():
        cfg.cuts = layer["CUT"]
    for k in ("NODES", "UINODE", "RPATH", "LDAPATH", "LUSER", "KRB_AUTH", "SPK_EXEC", "SPK_EXEC_MEM"):
        if k in layer:
            cfg.extra[k] = layer[k]
