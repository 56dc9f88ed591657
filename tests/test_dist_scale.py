"""Multi-rank EM at world sizes 4 and 8 (gloo on the CPU; the same code runs RCCL on GPUs),
the deterministic reduction mode (bitwise equal to one process emulating the shards) and the
strong-scaling bench path."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_dist import _free_port, _run  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world,exchange", [(4, "dense"), (4, "sparse"), (8, "dense"), (8, "sparse")])
def test_world_n_em_matches_single_rank(tmp_path, world, exchange):
    one = _run(1, str(tmp_path / "w1"), exchange)
    many = _run(world, str(tmp_path / f"w{world}"), exchange)
    L1, Ln = np.array(one[0][1]), np.array(many[0][1])
    assert L1.shape == Ln.shape
    assert np.allclose(L1, Ln, rtol=1e-10), (L1, Ln)
    for r in range(1, world):                                        # every rank: the same bits
        assert many[r][1] == many[0][1] and many[r][2] == many[0][2]
        assert np.array_equal(many[r][5], many[0][5])
    g1 = np.loadtxt(tmp_path / "w1" / "final.gamma")
    gn = np.loadtxt(tmp_path / f"w{world}" / "final.gamma")
    assert g1.shape == gn.shape and np.allclose(g1, gn, rtol=1e-6)
    assert np.allclose(one[0][5], many[0][5], rtol=1e-9, atol=1e-12)
    m = json.load(open(tmp_path / f"w{world}" / "lda_stats.json"))["metrics"]
    assert m["exchange_bytes_per_iter"] > 0 and m["exchange_seconds_per_iter"] > 0
    assert m["exchange"] == ("dense-allreduce" if exchange == "dense" else "sparse-alltoall")
    parts = np.concatenate([np.atleast_2d(np.loadtxt(tmp_path / f"w{world}" / f"{r}.gamma"))
                            for r in range(world) if (tmp_path / f"w{world}" / f"{r}.gamma").stat().st_size])
    assert np.allclose(parts, gn, atol=1e-9)


def _det_worker(rank, world, port, outdir, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), ONI_DIST_DETERMINISTIC="1")
    torch.set_num_threads(1)
    try:
        from oni_ml_amd.models.lda.estimate import estimate
        from oni_ml_amd.models.lda.settings import LDASettings
        from oni_ml_amd.parallel import dist as D
        from oni_ml_amd.synth.corpus import planted_corpus
        ctx = D.init_from_env(backend="gloo")
        assert ctx.deterministic
        c = planted_corpus(num_docs=240, num_terms=120, num_topics=4, seed=9)
        res = estimate(c, 6, 2.5, LDASettings(em_max_iter=4), "random", outdir, backend="torch", device="cpu",
                       dist=ctx, seed=1)
        q.put((rank, [x[0] for x in res.likelihoods], res.alpha, res.gamma, res.log_beta))
        ctx.shutdown()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None, None))


def test_deterministic_world4_bitwise_equals_emulated_shards(tmp_path):
    """ONI_DIST_DETERMINISTIC=1: four ranks give bitwise the model of one process emulating the
    same four shards (likelihoods, alpha, gamma, beta)."""
    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.synth.corpus import planted_corpus
    world, port = 4, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_det_worker, args=(r, world, port, str(tmp_path / "d4"), q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted([q.get(timeout=300) for _ in ps], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    for o in out:
        assert o[1] != "ERR", o[2]
    torch.set_num_threads(1)
    c = planted_corpus(num_docs=240, num_terms=120, num_topics=4, seed=9)
    eng = LDAEngine(c, 6, LDASettings(em_max_iter=4), backend="torch", device="cpu", seed=1, emulate_shards=world)
    r = eng.run()
    L = [x[0] for x in r.likelihoods]
    assert out[0][1] == L
    assert out[0][2] == eng.alpha
    # each rank returns its own gamma block (never gathered); in rank order they are the whole gamma
    assert np.array_equal(np.concatenate([o[3] for o in out]), eng.gather_gamma())
    assert np.array_equal(out[0][4], eng.log_beta())
    # without emulation the single process sums in another order: equal to rounding only
    eng1 = LDAEngine(c, 6, LDASettings(em_max_iter=4), backend="torch", device="cpu", seed=1)
    eng1.run()
    assert np.allclose(eng1.log_beta(), eng.log_beta(), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("world", [4, 8])
def test_bench_strong_scaling_cpu_rehearsal(world):
    """bench.py --scaling strong: one day, its documents sharded over the ranks (chain-aware,
    dist.engine_bounds: oni-lda-c's one model.dat over MPI ranks), value aggregated over all ranks."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus",
                        str(world), "--steps", "1", "--warmup", "1", "--events", "3000", "--device", "cpu",
                        "--scaling", "strong", "--converge", "0", "--e2e", "0", "--e2e-cold", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == world and out["scaling"] == "strong" and out["config"]["parallelism"] == f"dp{world}"
    assert out["value"] > 0


def test_bench_world8_gloo_shards_chain_and_weak_vocabulary():
    """bench.py at N = 8 over gloo (the RCCL code paths rehearsed on the CPU; no hardware claim):
    the strong-scaling shards tile the one-day corpus and are the engine's chain-aware cut
    (dist.engine_bounds: the longest document's rank carries no more than the cut's modelled share), and
    the weak run's union vocabulary (one day per rank, seeds 1000 r) equals a one-process union of the
    same eight days (reference: ml_ops.sh:73-80, one model.dat over the MPI ranks)."""
    import hashlib
    from oni_ml_amd.parallel.dist import chain_kappa, engine_bounds
    from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
    world, events = 8, 3000
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus",
                        str(world), "--steps", "1", "--warmup", "1", "--events", str(events), "--device", "cpu",
                        "--e2e", "0", "--e2e-cold", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=1200,
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == world and out["scaling"] == "strong"
    # strong: one corpus, its documents tiled by the ranks' contiguous shards -- the engine's cut
    c, _, _ = synthetic_flow_corpus(events=events, seed=0, device="cpu", return_names=True)
    sh = out["shards"]
    assert len(sh) == world and sh[0]["doc_range"][0] == 0 and sh[-1]["doc_range"][1] == c.num_docs
    assert all(sh[i]["doc_range"][1] == sh[i + 1]["doc_range"][0] for i in range(world - 1))
    assert sum(s["nnz"] for s in sh) == c.nnz
    assert [tuple(s["doc_range"]) for s in sh] == [tuple(b) for b in engine_bounds(c.doc_ptr, world, K=20)]
    lens = np.diff(c.doc_ptr)
    p = int(np.argmax(lens))
    rank_p = next(i for i, s in enumerate(sh) if s["doc_range"][0] <= p < s["doc_range"][1])
    assert sh[rank_p]["max_doc_len"] == int(lens[p])
    # the chain rule's cost of the longest document's rank is no worse than a plain nnz cut's
    others = sh[rank_p]["nnz"] - int(lens[p])
    kap = chain_kappa(20)
    plain = max(s["nnz"] for s in sh)
    assert kap * lens[p] + others <= max(kap * lens[p] + plain, plain) + 1e-9
    # weak: the union vocabulary of eight days equals the one-process union
    names = set()
    for rk in range(world):
        _, _, nm = synthetic_flow_corpus(events=events, seed=1000 * rk, device="cpu", return_names=True)
        names |= set(nm)
    union = sorted(names)
    assert out["weak_vocab"] == len(union)
    assert out["weak_vocab_sha16"] == hashlib.sha256("\n".join(union).encode()).hexdigest()[:16]
    assert out["weak_docs"] > c.num_docs
