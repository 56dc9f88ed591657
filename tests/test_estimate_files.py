"""Exact per-rank gamma blocks of a multi-rank run (estimate.load_final_rows): blocks are used only
when they form ONE run's complete tiling; leftovers of another run fall back to final.gamma's text."""
import os

import numpy as np

from oni_ml_amd.io import ldac
from oni_ml_amd.models.lda.estimate import _save_npz_atomic, load_final_rows


def _setup(tmp_path, D=10, K=4):
    rng = np.random.default_rng(0)
    g = rng.random((D, K)) + 0.5
    lb = np.log(rng.random((K, 7)) + 0.1)
    np.savez(os.path.join(tmp_path, "final_model.npz"), log_beta=lb, alpha=np.float64(0.3))
    ldac.save_gamma(os.path.join(tmp_path, "final.gamma"), g)
    return g, lb


def _rank_file(tmp_path, r, g, a, b, world, lik):
    _save_npz_atomic(os.path.join(tmp_path, f"final_gamma.rank{r}.npz"), gamma=g[a:b],
                     doc_range=np.asarray([a, b], np.int64), run=np.asarray([world, lik], np.float64))


def test_rank_blocks_exact(tmp_path):
    g, lb = _setup(str(tmp_path))
    _rank_file(str(tmp_path), 0, g, 0, 6, 2, -123.5)
    _rank_file(str(tmp_path), 1, g, 6, 10, 2, -123.5)
    rows, lb2 = load_final_rows(str(tmp_path), 3, 9)
    assert np.array_equal(rows, g[3:9])          # bitwise: not the %5.10f text
    assert np.array_equal(lb2, lb)
    assert not any(f.endswith(".tmp.npz") for f in os.listdir(tmp_path))


def test_stale_block_of_another_run_is_ignored(tmp_path):
    g, _ = _setup(str(tmp_path))
    stale = g + 1.0
    _rank_file(str(tmp_path), 0, g, 0, 6, 2, -123.5)
    _rank_file(str(tmp_path), 1, g, 6, 10, 2, -123.5)
    _rank_file(str(tmp_path), 2, stale, 6, 10, 3, -999.0)   # leftover of an earlier 3-rank run
    rows, _ = load_final_rows(str(tmp_path), 0, 10)
    assert np.array_equal(rows, g)


def test_incomplete_run_falls_back_to_text(tmp_path):
    g, _ = _setup(str(tmp_path))
    stale = g + 1.0
    _rank_file(str(tmp_path), 0, g, 0, 6, 2, -123.5)         # its partner is missing
    _rank_file(str(tmp_path), 1, stale, 3, 10, 3, -999.0)   # another run's block overlapping it
    rows, _ = load_final_rows(str(tmp_path), 0, 10)
    assert np.allclose(rows, g, atol=1e-9) and not np.array_equal(rows, stale[0:10])
    assert np.array_equal(rows, ldac.load_gamma(os.path.join(str(tmp_path), "final.gamma")))
