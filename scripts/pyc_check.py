#!/usr/bin/env python
"""Are the installed packages' cached bytecode files usable by this interpreter on this machine?

A .pyc is reused only if its header matches the source (magic, and the source's mtime and size for
timestamp pycs).  When they do not -- e.g. an image whose sources' mtimes changed after the pycs were
written, under a user who cannot rewrite them -- every fresh process compiles those modules again
(cold `ml_ops`: scripts/cold_start.py's cProfile shows it as builtins.compile).

  python scripts/pyc_check.py [torch numpy ...]
"""
import importlib.util
import json
import os
import sys


def check(pkg):
    spec = importlib.util.find_spec(pkg)
    root = os.path.dirname(spec.origin)
    ok = stale = missing = 0
    writable = os.access(os.path.join(root, "__pycache__"), os.W_OK)
    for dp, _, files in os.walk(root):
        for f in files:
            if not f.endswith(".py"):
                continue
            src = os.path.join(dp, f)
            pyc = importlib.util.cache_from_source(src)
            try:
                with open(pyc, "rb") as fh:
                    hdr = fh.read(16)
            except OSError:
                missing += 1
                continue
            st = os.stat(src)
            flags = int.from_bytes(hdr[4:8], "little")
            good = hdr[:4] == importlib.util.MAGIC_NUMBER and (
                flags != 0 or (int.from_bytes(hdr[8:12], "little") == int(st.st_mtime) & 0xFFFFFFFF
                               and int.from_bytes(hdr[12:16], "little") == st.st_size & 0xFFFFFFFF))
            ok += good
            stale += not good
    return dict(package=pkg, root=root, usable=ok, stale=stale, missing=missing, cache_writable=writable,
                pycache_prefix=sys.pycache_prefix)


if __name__ == "__main__":
    for p in sys.argv[1:] or ["torch", "numpy"]:
        print(json.dumps(check(p)))
