"""Document data parallelism over torch.distributed (gloo on the CPU; the same code runs RCCL on GPUs)."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oni_ml_amd.parallel.dist import shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, q, exchange="auto"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), ONI_DIST_EXCHANGE=exchange)
    torch.set_num_threads(1)
    try:
        from oni_ml_amd.parallel import dist as D
        from oni_ml_amd.models.lda.estimate import estimate
        from oni_ml_amd.models.lda.settings import LDASettings
        from oni_ml_amd.synth.corpus import planted_corpus
        ctx = D.init_from_env(backend="gloo")
        c = planted_corpus(num_docs=240, num_terms=120, num_topics=4, seed=9) if rank == 0 else None
        c = ctx.broadcast_corpus(c)
        if exchange == "sparse":
            # disjoint-ish vocabularies per shard (as IP/port words of different days): words of the
            # second half of the documents are shifted, so the shards share only a few words
            c = _shifted_vocab(c)
        res = estimate(c, 6, 2.5, LDASettings(em_max_iter=4), "random", outdir, backend="torch", device="cpu",
                       dist=ctx, seed=1, write_rank_gamma=True)
        g = ctx.gather_rows(np.full((rank + 1, 2), float(rank)), sum(range(1, world + 1)))
        q.put((rank, [x[0] for x in res.likelihoods], res.alpha, g.tolist(), res.gamma.shape, res.log_beta))
        ctx.shutdown()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, "ERR", traceback.format_exc(), None, None, None))


def _shifted_vocab(c):
    """Documents of the second half use word ids shifted by V (plus every 10th word kept shared)."""
    from oni_ml_amd.corpus.csr import Corpus
    w = c.word_idx.copy()
    half = c.doc_ptr[c.num_docs // 2]
    tail = w[half:]
    w[half:] = np.where(tail % 10 == 0, tail, tail + c.num_terms)
    return Corpus(c.doc_ptr.copy(), w, c.counts.copy(), 2 * c.num_terms)


def _run(world, outdir, exchange="auto"):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, outdir, q, exchange)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    out.sort(key=lambda x: x[0])
    for o in out:
        assert o[1] != "ERR", o[2]
    return out


def test_shard_bounds_balanced_and_contiguous():
    ptr = np.concatenate([[0], np.cumsum(np.r_[np.full(90, 1), [500], np.full(9, 3)])])
    b = shard_bounds(ptr, 4)
    assert b[0][0] == 0 and b[-1][1] == 100 and all(b[i][1] == b[i + 1][0] for i in range(3))


@pytest.mark.parametrize("exchange", ["dense", "sparse"])
def test_two_rank_em_matches_single_rank(tmp_path, exchange):
    """dense: ring all-reduce of class_word; sparse: VocabExchange all-to-all of the shared rows."""
    one = _run(1, str(tmp_path / "w1"), exchange)
    two = _run(2, str(tmp_path / "w2"), exchange)
    L1, L2 = np.array(one[0][1]), np.array(two[0][1])
    assert L1.shape == L2.shape
    assert np.allclose(L1, L2, rtol=1e-10), (L1, L2)             # all-reduce order only
    assert two[0][1] == two[1][1] and two[0][2] == two[1][2]       # ranks agree exactly
    assert two[0][3] == [[0.0, 0.0], [1.0, 1.0], [1.0, 1.0]]      # order-preserving row gather
    g1 = np.loadtxt(tmp_path / "w1" / "final.gamma")
    g2 = np.loadtxt(tmp_path / "w2" / "final.gamma")
    assert g1.shape == g2.shape and np.allclose(g1, g2, rtol=1e-6)
    # the full model (final.beta) agrees: the sparse exchange rebuilds the non-local rows for saves
    assert np.allclose(one[0][5], two[0][5], rtol=1e-9, atol=1e-12)
    assert np.array_equal(two[0][5], two[1][5])
    # per-rank gamma blocks concatenate to final.gamma (README.md:121)
    parts = np.concatenate([np.atleast_2d(np.loadtxt(tmp_path / "w2" / f"{r}.gamma")) for r in range(2)])
    assert np.allclose(parts, g2, atol=1e-9)
    # per-rank <rank>.beta: log of the rank's own class_word over the global totals, so the ranks'
    # probabilities sum to final.beta's
    from oni_ml_amd.io import ldac
    fb = ldac.load_beta(str(tmp_path / "w2" / "final.beta"))
    rb = [ldac.load_beta(str(tmp_path / "w2" / f"{r}.beta")) for r in range(2)]
    assert all(b.shape == fb.shape for b in rb)
    comb = np.log(np.exp(rb[0]) + np.exp(rb[1]))
    live = fb > -99
    assert live.any() and np.allclose(comb[live], fb[live], atol=1e-8)
    if exchange == "sparse":   # disjoint-ish vocabularies: each rank misses words the other has
        assert (rb[0] == -100).sum() > 0 and (rb[1] == -100).sum() > 0


def test_bench_two_rank_cpu_rehearsal():
    """bench.py at N = 2 on gloo: every field of the BENCH line -- the strong-scaling 1-day value (one
    corpus sharded over the ranks), the weak-scaling secondary, the row-sharded ml_ops pipeline in-process
    (warm) and as fresh child processes (cold)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                        "--steps", "1", "--warmup", "1", "--events", "5000", "--device", "cpu"],
                       cwd=root, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["value"] > 0
    assert out["scaling"] == "strong" and out["config"]["docs"] == out["config"]["global_batch"]
    # the strong run splits ONE corpus: the shards partition its documents
    sh = out["shards"]
    assert sh[0]["doc_range"][0] == 0 and sh[0]["doc_range"][1] == sh[1]["doc_range"][0]
    assert sh[1]["doc_range"][1] == out["config"]["docs"]
    assert sum(s["nnz"] for s in sh) == out["config"]["nnz"]
    assert out["weak_docs_per_sec"] > 0 and out["weak_docs"] > out["config"]["docs"]
    for k in ("e2e_wall_s", "e2e_cold_wall_s"):
        assert out[k] > 0, k
    assert out["e2e_cold_wall_s"] >= out["e2e_cold_inprocess_wall_s"] > 0
    assert set(out["e2e_stage_s"]) >= {"load", "flow_pre", "lda_pre", "lda", "lda_post", "flow_post"}


@pytest.mark.parametrize("exchange", ["dense", "sparse"])
def test_two_rank_ml_ops_pipeline_matches_one_rank(tmp_path, exchange):
    """`ml_ops` under torchrun with 2 ranks (gloo, torch backend): rank 0 featurizes and broadcasts the
    corpus, the ranks share the LDA stage (dense all-reduce or sparse all-to-all of class_word rows),
    rank 0 exports and scores.  The output files match a single-rank run."""
    import subprocess
    import sys
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.synth.flow import generate_flow_day
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    generate_flow_day(str(tmp_path / "in") + "/", events=3000, seed=2, n_internal=200, n_external=300)
    st = tmp_path / "settings.txt"
    st.write_text(LDASettings(em_max_iter=3).dumps())
    env = dict(os.environ, ONI_CONF=str(tmp_path / "none.conf"), ONI_DIST_EXCHANGE=exchange)
    args = ["ml_ops", "20160122", "flow", "1e-3", "--flow-path", str(tmp_path / "in"), "--backend", "torch",
            "--settings", str(st), "--threads", "2", "--quiet"]
    r1 = subprocess.run([sys.executable, "-m", "oni_ml_amd"] + args + ["--lpath", str(tmp_path / "one")], cwd=root,
                        capture_output=True, text=True, env=env, timeout=600)
    assert r1.returncode == 0, r1.stderr[-2000:]
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                         "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "oni_ml_amd"] + args +
                        ["--lpath", str(tmp_path / "two"), "--gpus", "2"], cwd=root, capture_output=True, text=True,
                        env=env, timeout=600)
    assert r2.returncode == 0, r2.stderr[-3000:]
    for f in ("doc.dat", "words.dat", "model.dat"):
        assert (tmp_path / "one" / f).read_text() == (tmp_path / "two" / f).read_text(), f
    g1, g2 = np.loadtxt(tmp_path / "one" / "final.gamma"), np.loadtxt(tmp_path / "two" / "final.gamma")
    assert g1.shape == g2.shape and np.allclose(g1, g2, rtol=1e-6, atol=1e-7)
    b1, b2 = np.loadtxt(tmp_path / "one" / "final.beta"), np.loadtxt(tmp_path / "two" / "final.beta")
    assert np.allclose(b1, b2, rtol=1e-8, atol=1e-9)
    l1 = [l.split("\t")[0] for l in (tmp_path / "one" / "likelihood.dat").read_text().splitlines()]
    l2 = [l.split("\t")[0] for l in (tmp_path / "two" / "likelihood.dat").read_text().splitlines()]
    assert np.allclose(np.array(l1, float), np.array(l2, float), rtol=1e-10)
    s1 = json.load(open(tmp_path / "one" / "run_summary.json"))
    s2 = json.load(open(tmp_path / "two" / "run_summary.json"))
    assert s1["scored"] == s2["scored"] > 0
    # the same events flagged, in the same order; the two scores agree up to the all-reduce order
    f1 = (tmp_path / "one" / "flow_results.csv").read_text().splitlines()[:20]
    f2 = (tmp_path / "two" / "flow_results.csv").read_text().splitlines()[:20]
    assert len(f1) == len(f2)
    for a, b in zip(f1, f2):
        ra, rb = a.split(","), b.split(",")
        assert ra[:-2] == rb[:-2]
        assert np.allclose([float(x) for x in ra[-2:]], [float(x) for x in rb[-2:]], rtol=1e-9)


def test_chain_bounds_isolate_the_longest_document():
    """Chain-aware shards: contiguous, cover every document once, the longest document alone on its
    rank, the rest nnz-balanced on both sides; nnz balance when no chain dominates."""
    from oni_ml_amd.parallel.dist import chain_bounds
    rng = np.random.default_rng(4)
    lens = rng.integers(1, 12, 5000)
    lens[3100] = 4000                                   # 4000 x 88 >> nnz / 8
    ptr = np.concatenate([[0], np.cumsum(lens)])
    for world in (3, 4, 8):
        b = chain_bounds(ptr, world)
        assert len(b) == world and b[0][0] == 0 and b[-1][1] == 5000
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        assert (3100, 3101) in b
        others = [int(ptr[e] - ptr[s]) for s, e in b if (s, e) != (3100, 3101)]
        assert max(others) < 1.3 * (ptr[-1] - 4000) / (world - 1)
    flat = np.concatenate([[0], np.cumsum(np.full(1000, 5))])
    assert chain_bounds(flat, 4) == shard_bounds(flat, 4)
    edge = np.concatenate([[0], np.cumsum(np.r_[9000, np.full(999, 5)])])   # longest first
    b = chain_bounds(edge, 4)
    assert b[0] == (0, 1) and b[-1][1] == 1000 and len(b) == 4


def test_engine_bounds_balance_modelled_cost_not_entries():
    """The engine's cut balances the modelled E-step cost (dist.doc_costs: entries weighted by length class,
    fitted to the config-5 shards), not entries: ranks of long documents (all 20 sweeps) take fewer entries
    than ranks of short ones; at K > 32 a split document's chain is capped (SPLIT_CHAIN_NS)."""
    from oni_ml_amd.parallel.dist import SPLIT_CHAIN_NS, chain_ns, doc_costs, engine_bounds
    rng = np.random.default_rng(1)
    lens = np.r_[rng.integers(2100, 5000, 400), rng.integers(5, 200, 20000)]
    ptr = np.concatenate([[0], np.cumsum(lens)])
    b = engine_bounds(ptr, 4, K=100)
    cost = doc_costs(lens, 100)
    per_cost = [cost[s:e].sum() for s, e in b]
    per_nnz = [int(ptr[e] - ptr[s]) for s, e in b]
    assert max(per_cost) < 1.05 * sum(per_cost) / 4                   # cost-balanced
    assert per_nnz[0] < 0.8 * per_nnz[-1]                              # the long-document rank: fewer entries
    assert chain_ns(443_000, 100) == SPLIT_CHAIN_NS < chain_ns(443_000, 20)
    assert doc_costs(np.array([4, 5, 256, 257, 2048, 2049]), 100).tolist() == pytest.approx(
        [4 * 2.27, 5 * 1.30, 256 * 1.30, 257 * 1.79, 2048 * 1.79, 2049 * 3.17])
