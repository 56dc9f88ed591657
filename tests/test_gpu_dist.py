"""Multi-rank HIP EM on one GPU (gloo rehearsal of the RCCL path): dense all-reduce and the
sparse all-to-all class_word exchange give the single-rank trajectory."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, exchange, overlap="1"):
    env = dict(os.environ, ONI_DIST_EXCHANGE=exchange, ONI_DIST_BACKEND="gloo", ONI_DIST_OVERLAP=overlap)
    if world == 1:
        cmd = [sys.executable, "scripts/dist_check.py"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "scripts/dist_check.py"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_two_rank_hip_exchanges_match_single_rank():
    one = _run(1, "auto")
    dense = _run(2, "dense")
    sparse = _run(2, "sparse")                 # shared rows in flight during the private suff-stats
    sparse_seq = _run(2, "sparse", overlap="0")
    assert one["exchange"] == "none" and dense["exchange"] == "dense-allreduce"
    assert sparse["exchange"] == "sparse-alltoall" and 0 < sparse["rows"] < 4000
    assert sparse_seq["likelihoods"] == sparse["likelihoods"]      # same arithmetic, other schedule
    for o in (dense, sparse):
        assert len(o["likelihoods"]) == len(one["likelihoods"])
        assert np.allclose(o["likelihoods"], one["likelihoods"], rtol=2e-6), (o["likelihoods"], one["likelihoods"])
        assert o["gamma_shape"] == one["gamma_shape"]
        assert abs(o["gamma_sum"] - one["gamma_sum"]) / one["gamma_sum"] < 1e-5
        assert abs(o["beta_checksum"] - one["beta_checksum"]) / abs(one["beta_checksum"]) < 1e-5
