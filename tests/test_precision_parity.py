"""scripts/precision_parity.py: the engine-comparison harness behind profiles/r1_precision_parity.md.

CPU: the two fp64 engines (PyTorch Jacobi, literal lda-c Gauss-Seidel) on a small synthetic day; the
harness must report the pairwise metrics in range and write both outputs.
GPU: the fp64 HIP engine against the C++ engine with the same block schedule."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "precision_parity.py")


def _run(tmp_path, engines, events):
    out = tmp_path / "parity.json"
    # one host thread per engine: torch's OpenMP workers spin-wait, and beside other busy processes
    # (pytest -n, a parity run) an 8-thread pool on this tiny corpus ran ~60x slower than one thread
    env = dict(os.environ, OMP_NUM_THREADS="1", ONI_THREADS="1")
    r = subprocess.run([sys.executable, SCRIPT, "--events", str(events), "--engines", engines, "--json", str(out),
                        "--md", str(tmp_path / "parity.md")], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(out.read_text())


def test_parity_harness_fp64_engines(tmp_path):
    res = _run(tmp_path, "torch,cpu", 8000)
    e = res["engines"]
    assert set(e) == {"torch", "cpu"} and set(res["pairs"]) == {"torch vs cpu"}
    p = res["pairs"]["torch vs cpu"]
    assert 0.0 <= p["final_likelihood_rel_diff"] < 1e-2
    assert 0.5 < p["score_spearman"] <= 1.0
    assert 0.0 <= p["lowest_0p1pct_overlap"] <= 1.0
    for v in e.values():
        assert v["final_likelihood"] < 0 and v["alpha"] > 0 and len(v["likelihood_trajectory"]) == v["em_iterations"]
    assert (tmp_path / "parity.md").read_text().startswith("# Precision / schedule parity")


def test_parity_harness_block_schedule_cpu(tmp_path):
    """The C++ engine with the GPU engine's block schedule (cpuU) against literal lda-c (cpu): the
    block schedule is the GPU engine's oracle, so its distance to lda-c is the GPU engine's."""
    p = _run(tmp_path, "cpuU,cpu", 8000)["pairs"]["cpuU vs cpu"]
    assert p["final_likelihood_rel_diff"] < 1e-3
    assert p["alpha_rel_diff"] < 0.05


@pytest.mark.gpu
def test_fp64_hip_engine_tracks_block_oracle(tmp_path):
    """fp64 GPU engine vs the C++ engine with the same block schedule: the same model, trained to
    convergence (float64 on both sides)."""
    p = _run(tmp_path, "hip,cpuU", 50000)["pairs"]["hip vs cpuU"]
    assert p["likelihood_rel_diff_max"] < 1e-8
    assert p["alpha_rel_diff"] < 1e-7
    assert p["theta_doc_argmax_agree"] > 0.999
    assert p["lowest_0p1pct_overlap"] > 0.99
