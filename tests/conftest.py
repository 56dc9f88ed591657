import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _ensure_built():
    """Fresh checkouts carry no .so files (git-ignored): build the native runtime (and the gfx950
    kernels when hipcc is present) once, in-tree, before the first test imports them."""
    from oni_ml_amd import _build

    try:
        _build.build_all(verbose=False, hip=os.path.exists(_build.HIPCC), native=True)
    except Exception as e:  # surfaced by the tests that need the extension
        print(f"[conftest] native build failed: {e}")


def pytest_configure(config):
    _ensure_built()
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def hip():
    """The HIP op wrappers; on a GPU box a missing extension is an error, not a skip."""
    from oni_ml_amd.ops import hip as H

    H.lib()  # raises loudly if _onihip is missing
    return H
