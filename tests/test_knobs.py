"""Every ONI_* environment variable the source reads is registered in oni_ml_amd/knobs.py (at most 20,
each documented there and in docs/KNOBS.md): round 5 removed the A/B switches of variants measured slower."""
import os
import re

from oni_ml_amd import knobs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = ("oni_ml_amd", "csrc", "scripts", "bench.py", "__graft_entry__.py")
NOT_KNOBS = {"ONI_KS", "ONI_HIP_CHECK", "ONI_FOR_EACH_KS"}      # C++ macros


def _named():
    names = set()
    for top in SOURCES:
        p = os.path.join(ROOT, top)
        files = [p] if os.path.isfile(p) else [os.path.join(d, f) for d, _, fs in os.walk(p) for f in fs]
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp", ".sh")) and "__pycache__" not in f:
                names |= set(re.findall(r"\bONI_[A-Z0-9_]+", open(f, encoding="utf-8", errors="replace").read()))
    return names - NOT_KNOBS


def test_every_knob_is_registered():
    unknown = sorted(_named() - set(knobs.KNOBS))
    assert not unknown, unknown


def test_knob_budget_and_docs():
    assert len(knobs.KNOBS) <= 20
    assert all(len(doc) > 20 for doc in knobs.KNOBS.values())
    table = open(os.path.join(ROOT, "docs", "KNOBS.md"), encoding="utf-8").read()
    listed = set(re.findall(r"^\| `(ONI_[A-Z0-9_]+)` \|", table, re.M))
    assert listed == set(knobs.KNOBS)


def test_unregistered_knob_refused():
    import pytest
    with pytest.raises(KeyError):
        knobs.get("ONI_NOT_A_KNOB")
