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
    # overlap "0": the sparse exchange not overlapped with the private words' suff-stats (sparse-serial)
    mode = "sparse-serial" if (exchange == "sparse" and overlap == "0") else exchange
    env = dict(os.environ, ONI_DIST_EXCHANGE=mode, ONI_DIST_BACKEND="gloo")
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
    # same arithmetic, other schedule; the document-likelihood sum is sliced over the grid of the
    # launch that carries it (plan A vs the whole vocabulary), so only its last bits may differ
    assert np.allclose(sparse_seq["likelihoods"], sparse["likelihoods"], rtol=1e-13, atol=0)
    for o in (dense, sparse):
        assert len(o["likelihoods"]) == len(one["likelihoods"])
        assert np.allclose(o["likelihoods"], one["likelihoods"], rtol=2e-6), (o["likelihoods"], one["likelihoods"])
        assert o["gamma_shape"] == one["gamma_shape"]
        assert abs(o["gamma_sum"] - one["gamma_sum"]) / one["gamma_sum"] < 1e-5
        assert abs(o["beta_checksum"] - one["beta_checksum"]) / abs(one["beta_checksum"]) < 1e-5


@pytest.mark.parametrize("exchange", ["dense", "sparse"])
def test_four_rank_fp64_engine_matches_single_rank(exchange):
    """The fp64 block Gauss-Seidel engine on 4 ranks (one GPU, gloo): per-document E-steps are
    shard-independent, so only the order of the cross-rank sums differs from one rank."""
    one = _run(1, "auto")
    four = _run(4, exchange)
    assert four["world"] == 4 and four["precision"] == "fp64"
    assert len(four["likelihoods"]) == len(one["likelihoods"])
    assert np.allclose(four["likelihoods"], one["likelihoods"], rtol=1e-10, atol=0)
    assert abs(four["alpha"] - one["alpha"]) / one["alpha"] < 1e-9
    assert abs(four["gamma_sum"] - one["gamma_sum"]) / one["gamma_sum"] < 1e-10
    assert abs(four["beta_checksum"] - one["beta_checksum"]) / abs(one["beta_checksum"]) < 1e-10


def test_rows_accumulate_kernel_matches_rank_order_sum():
    """HIP rows_accumulate (VocabExchange.accumulate's one-launch form) == fill + index_add per
    source in rank order, bit for bit (fp64 adds in the same order), and the engine's
    VocabExchange.accumulate issues exactly that one launch for fp64 statistics."""
    import torch
    from oni_ml_amd.ops import hip as H
    g = torch.Generator().manual_seed(3)
    V, W, world, me = 5000, 20, 4, 2
    mine = torch.unique(torch.randint(0, V, (1800,), generator=g))
    own = torch.rand(V, W, generator=g, dtype=torch.float64)
    commons, recv_parts = [], []
    for s in range(world):
        if s == me:
            commons.append(torch.zeros(0, dtype=torch.int64))
            continue
        c = mine[torch.rand(mine.numel(), generator=g) < 0.4]
        commons.append(c)
        recv_parts.append(torch.rand(c.numel(), W, generator=g, dtype=torch.float64))
    recv = torch.cat(recv_parts)
    offsets = np.concatenate([[0], np.cumsum([c.numel() for c in commons])]).tolist()
    # reference: fill + index_add in rank order
    ref = torch.full((V, W), 7.0, dtype=torch.float64)
    ref.index_fill_(0, mine, 0)
    for s in range(world):
        if s == me:
            ref.index_add_(0, mine, own.index_select(0, mine))
        elif commons[s].numel():
            ref.index_add_(0, commons[s], recv[offsets[s]:offsets[s + 1]])
    # CSR plan as VocabExchange builds it
    rows, keys, srcs = [], [], []
    for s in range(world):
        if s == me:
            rr, ss = torch.arange(mine.numel()), torch.full((mine.numel(),), -1)
        else:
            rr, ss = torch.searchsorted(mine, commons[s]), offsets[s] + torch.arange(commons[s].numel())
        rows.append(rr), keys.append(rr * world + s), srcs.append(ss)
    order = torch.argsort(torch.cat(keys), stable=True)
    rs, src = torch.cat(rows)[order], torch.cat(srcs)[order]
    ptr = torch.zeros(mine.numel() + 1, dtype=torch.int64)
    ptr[1:] = torch.cumsum(torch.bincount(rs, minlength=mine.numel()), 0)
    d = torch.device("cuda")
    out = torch.full((V, W), 7.0, device=d, dtype=torch.float64)
    H.rows_accumulate(mine.to(d, torch.int32), ptr.to(d, torch.int32), src.to(d, torch.int32), own.to(d),
                      recv.to(d), out)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)
    # the engine path: VocabExchange.accumulate on fp64 device statistics is that one launch
    from oni_ml_amd.parallel.dist import VocabExchange
    x = VocabExchange.__new__(VocabExchange)
    x.width, x.local_rows32, x.acc_ptr, x.acc_src = W, mine.to(d, torch.int32), ptr.to(d, torch.int32), src.to(d, torch.int32)
    x.recv = recv.to(d)
    calls = []
    real = H.rows_accumulate
    H.rows_accumulate = lambda *a: (calls.append(1), real(*a))
    try:
        out2 = torch.full((V, W), 7.0, device=d, dtype=torch.float64)
        x.accumulate(out2, own.to(d))
    finally:
        H.rows_accumulate = real
    torch.cuda.synchronize()
    assert len(calls) == 1 and torch.equal(out2.cpu(), ref)


def _nccl_env(**kw):
    env = dict(os.environ, ONI_DIST_FORCE_GROUP="1", ONI_DIST_BACKEND="nccl", WORLD_SIZE="1", RANK="0",
               LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    env.update(kw)
    return env


@pytest.mark.parametrize("exchange,overlap", [("dense", "1"), ("sparse", "1"), ("sparse", "0")])
def test_nccl_one_rank_engine_matches_plain_run(exchange, overlap):
    """A one-rank RCCL process group (ONI_DIST_FORCE_GROUP=1) drives the engine's distributed path on
    the one-GPU box: init_process_group(device_id), the start-up self-check (all_reduce,
    barrier(device_ids), all_to_all_single), the E-step graph -> fp64 all-reduce of
    [likelihood, alpha_ss, class_total] -> (dense class_word all-reduce | sparse VocabExchange
    all-to-all, async when overlapped) -> M-step graph.  A sum over one rank is the identity, so the
    trajectory equals the plain single-process run."""
    one = _run(1, "auto")
    r = subprocess.run([sys.executable, "scripts/dist_check.py"], cwd=ROOT, capture_output=True, text=True,
                       timeout=300, env=_nccl_env(ONI_DIST_EXCHANGE="sparse-serial" if (exchange == "sparse" and
                                                                                       overlap == "0") else exchange))
    assert r.returncode == 0, r.stderr[-4000:]
    o = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert o["world"] == 1
    assert o["exchange"] == ("dense-allreduce" if exchange == "dense" else "sparse-alltoall")
    if exchange == "sparse" and overlap == "1":
        # the overlap mode sums the per-document likelihood / alpha_ss over the grid of its second
        # suff-stats launch (no shared words at one rank): the same terms in another association
        assert np.allclose(o["likelihoods"], one["likelihoods"], rtol=1e-13, atol=0)
        assert abs(o["alpha"] - one["alpha"]) <= 1e-12 * one["alpha"]
        assert abs(o["beta_checksum"] - one["beta_checksum"]) <= 1e-11 * abs(one["beta_checksum"])
        return
    assert o["likelihoods"] == one["likelihoods"]
    assert o["alpha"] == one["alpha"] and o["beta_checksum"] == one["beta_checksum"]
    assert o["gamma_sum"] == one["gamma_sum"]


def test_nccl_one_rank_sharded_pipeline_bytes_equal_single_process(tmp_path):
    """The row-sharded ml_ops pipeline (pipeline/sharded.py) over a one-rank RCCL group -- every
    shardio collective (all_gather, all_to_all_single, broadcast, barriers) on device buffers --
    writes byte for byte the files of the single-process pipeline."""
    from oni_ml_amd.synth.flow import generate_flow_day
    generate_flow_day(str(tmp_path / "in") + "/", events=200_000, seed=5)
    files = ["words.dat", "doc.dat", "model.dat", "final.beta", "final.gamma", "likelihood.dat", "doc_results.csv",
             "word_results.csv", "flow_results.csv", "word-assignments.dat"]
    outs = {}
    for mode in ("plain", "rccl"):
        lp = tmp_path / mode
        cmd = [sys.executable, "-m", "oni_ml_amd.cli", "ml_ops", "20160122", "flow", "1e-5", "--lpath", str(lp),
               "--flow-path", str(tmp_path / "in"), "--conf", "/nonexistent", "--quiet"]
        env = _nccl_env() if mode == "rccl" else dict(os.environ)
        r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-4000:]
        outs[mode] = json.load(open(lp / "run_summary.json"))
    assert outs["plain"]["scored"] == outs["rccl"]["scored"] > 0
    recs = [json.loads(l) for l in (tmp_path / "rccl" / "metrics.jsonl").read_text().splitlines()]
    assert any(x.get("stage") == "lda" and x.get("exchange") == "dense-allreduce" for x in recs)
    for f in files:
        assert (tmp_path / "plain" / f).read_bytes() == (tmp_path / "rccl" / f).read_bytes(), f
