"""Loader for the C++ host runtime module `_oninative` (CSV parser, formatters, lda-c reference)."""
from __future__ import annotations

import importlib
import os
import sys

_LIB = None
_ERR = None


def lib():
    global _LIB, _ERR
    if _LIB is None:
        here = os.path.join(os.path.dirname(os.path.dirname(__file__)), "_lib")
        if here not in sys.path:
            sys.path.insert(0, here)
        try:
            _LIB = importlib.import_module("_oninative")
        except Exception as e:
            _ERR = e
            raise RuntimeError(
                f"oni_ml_amd native runtime (_oninative) is not built or failed to load: {e!r}. "
                "Run `python -m oni_ml_amd._build`.") from e
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except RuntimeError:
        return False
