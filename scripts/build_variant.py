#!/usr/bin/env python
"""Build a variant of the `_onihip` extension with extra -D flags on csrc/hip/lda_gs64.hip, into its own
directory (A/B runs on the GPU box copy the tree and drop the variant's .so into oni_ml_amd/_lib):

  python scripts/build_variant.py abvar/r1 -DTEAM4_RMAX=1
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oni_ml_amd import _build as B  # noqa: E402


def main():
    outdir = Path(sys.argv[1]).resolve()
    defs = sys.argv[2:]
    outdir.mkdir(parents=True, exist_ok=True)
    hdrs = sorted((B.CSRC / "hip").glob("*.h"))
    objs = []
    for src in sorted((B.CSRC / "hip").glob("*.hip")) + [B.CSRC / "hip" / "bind_hip.cpp"]:
        if src.name == "lda_gs64.hip":
            o = outdir / "obj" / (src.stem + ".o")
            B._compile(src, o, [B.HIPCC], B.hip_flags() + defs, hdrs, True)
        else:
            o = B.OBJ / "hip" / (src.stem + ".o")     # the main build's object (python -m oni_ml_amd._build first)
            assert o.exists(), o
        objs.append(o)
    out = outdir / ("_onihip" + B._ext_suffix())
    B._link(out, objs, [B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-fPIC", "-o", str(out)] + [str(o) for o in objs],
            True)
    print(out)


if __name__ == "__main__":
    main()
