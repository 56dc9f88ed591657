"""A per-user bytecode cache when the installed packages' own cannot be used.

Python reuses a module's cached bytecode only if the .pyc header matches the source's mtime and size.
On the MI355X boxes the image's torch / numpy .pyc files are all stale against their sources (another
mtime after the image was assembled) and the non-root user cannot rewrite them (scripts/pyc_check.py:
torch 0 of 2,113 usable), so every fresh process compiled ~900 modules again: `import torch` 1.45-1.54 s,
against 0.69 s from a valid cache (profiles/r4_cold_start.md).  `ml_ops` is a fresh process per day
(ml_ops.sh:57,67,80,84,108), so it pays that every run.

``enable()`` -- called by ``python -m oni_ml_amd`` before anything imports torch -- points
``sys.pycache_prefix`` at ``$XDG_CACHE_HOME/oni_ml_amd/pycache`` (``~/.cache/...``) when the
site-packages holding torch is not writable.  The first process fills it; later ones load from it.
Validity is still checked against every source's mtime and size, exactly as for __pycache__, so an
upgraded package recompiles.  PYTHONPYCACHEPREFIX (the interpreter's own switch) wins when set;
ONI_PYCACHE=0 disables.
"""
from __future__ import annotations

import importlib.util
import os
import sys


def cache_dir() -> str:
    base = os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache")
    return os.path.join(base, "oni_ml_amd", "pycache")


def enable() -> str | None:
    """Set sys.pycache_prefix if needed; returns the prefix in use (None: the packages' own caches)."""
    if sys.pycache_prefix or os.environ.get("ONI_PYCACHE", "1") == "0" or sys.dont_write_bytecode:
        return sys.pycache_prefix
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.origin:
        return None
    if os.access(os.path.join(os.path.dirname(spec.origin), "__pycache__"), os.W_OK):
        return None                      # the installed caches are refreshed in place when stale
    d = cache_dir()
    try:
        os.makedirs(d, exist_ok=True)
    except OSError:
        return None
    if not os.access(d, os.W_OK):
        return None
    sys.pycache_prefix = d
    return d
