"""lda-c run settings (settings.txt) and model-level constants.

settings.txt (read by oni-lda-c's read_settings, called from ml_ops.sh:80) is
five lines::

    var max iter 20
    var convergence 1e-6
    em max iter 100
    em convergence 1e-4
    alpha estimate

The values above are upstream lda-c's shipped defaults (the
oni-lda-c copy is absent from the reference mount, so they are unverified).
lda-c stores both convergence thresholds as C ``float``; we keep that rounding.
"""
from __future__ import annotations

import re
from dataclasses import dataclass

import numpy as np

LAG = 5                  # save period of %03d.{beta,gamma,other}
NEWTON_THRESH = 1e-5     # alpha Newton stopping |df|
MAX_ALPHA_ITER = 1000
NUM_INIT = 1             # documents per topic for "seeded" init
LOG_FLOOR = -100.0       # lda_mle floor for class_word == 0


@dataclass
class LDASettings:
    var_max_iter: int = 20
    var_converged: float = 1e-6
    em_max_iter: int = 100
    em_converged: float = 1e-4
    estimate_alpha: bool = True
    # Engine schedule (not a settings.txt line): 0 = lda-c's per-word Gauss-Seidel;
    # U > 0 = block Gauss-Seidel with at most U gamma refreshes per sweep (lda_ref.cpp).
    gs_updates: int = 0
    # Period of the %03d.{beta,gamma,other} files and checkpoint (lda-c's compile-time LAG); 0 = only
    # 000 and final.  Not a settings.txt line: large runs (BASELINE config 5's ~8 GB gamma per save)
    # turn it down from the caller.
    lag: int = LAG

    def __post_init__(self):
        # lda-c keeps these as float32
        self.var_converged = float(np.float32(self.var_converged))
        self.em_converged = float(np.float32(self.em_converged))

    @staticmethod
    def parse(text: str) -> "LDASettings":
        def grab(key, cast, default):
            m = re.search(rf"^\s*{key}\s+(\S+)", text, re.MULTILINE)
            return cast(m.group(1)) if m else default

        alpha = grab("alpha", str, "estimate")
        return LDASettings(
            var_max_iter=grab("var max iter", int, 20),
            var_converged=grab("var convergence", float, 1e-6),
            em_max_iter=grab("em max iter", int, 100),
            em_converged=grab("em convergence", float, 1e-4),
            estimate_alpha=(alpha != "fixed"),
        )

    @staticmethod
    def load(path) -> "LDASettings":
        with open(path) as f:
            return LDASettings.parse(f.read())

    def dumps(self) -> str:
        return (f"var max iter {self.var_max_iter}\nvar convergence {self.var_converged:g}\n"
                f"em max iter {self.em_max_iter}\nem convergence {self.em_converged:g}\n"
                f"alpha {'estimate' if self.estimate_alpha else 'fixed'}\n")
