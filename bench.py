#!/usr/bin/env python
"""Headline benchmark: LDA variational-EM throughput on a synthetic 1-day netflow corpus.

Metric (BASELINE.json): "LDA docs/sec to convergence + ml_ops.sh wall-clock, 1-day netflow".

One step = one full EM iteration of the oni-lda-c algorithm: the length-bucketed
fused E-step run to per-document convergence (hipGraph replay), deterministic
sufficient statistics, RCCL all-reduce of class_word when N > 1, M-step and
the alpha Newton step.  value = documents processed per second summed over
all ranks (docs x timed EM iterations / max-over-ranks wall time).

Engine: the fp64 block Gauss-Seidel engine (--precision fp64, the default: lda-c's double
arithmetic and its per-word schedule up to blocks of ceil(n/32) words, csrc/hip/lda_gs64.hip);
--precision fp32 runs the experimental fp32 Jacobi engine (a known model bias against lda-c,
profiles/r2_precision_parity.md; its tests run only with ONI_EXPERIMENTAL=1).

value = LDA docs/s TO CONVERGENCE: a fresh random-init run trained until lda-c's EM loop test
stops it (device-side test, every iteration in full), docs x EM iterations / wall time, summed
over ranks.  The timed K-step window (``ms_per_step``: W untimed warm-up iterations, then exactly
K EM iterations bracketed by barrier + synchronize, max over ranks) is reported beside it as
``window_docs_per_sec``.

--scaling weak (default): rank r featurizes its own synthetic netflow day (1M events, seed r)
through the real pipeline (CSV -> C++ ingest -> GPU featurization -> corpus), the ranks agree on
the union vocabulary, and the N days are trained as one N-day corpus with documents sharded by
rank.  --scaling strong: every rank builds the SAME day and the engine shards its documents
nnz-balanced over the N ranks, as oni-lda-c splits one model.dat over its MPI ranks
(ml_ops.sh:22-23,80).  Weights are random-init (lda-c "random" start).  Extra (N = 1): the
wall-clock of the whole ml_ops flow pipeline on the day, with a TOL that flags >= 10^4 events.

  python bench.py --gpus N --steps K --warmup W
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)
  CPU rehearsal of the multi-rank path: --device cpu (gloo, torch backend).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "LDA docs/sec to convergence + ml_ops.sh wall-clock, 1-day netflow"


def _baseline():
    try:
        with open(os.path.join(ROOT, "BASELINE.json")) as f:
            b = json.load(f)
        v = b.get("measured_baseline", {}).get("lda_docs_per_sec")
        return float(v) if v else None
    except Exception:
        return None


def build_corpus(args, rank, ctx, dev):
    seed = args.seed + (1000 * rank if args.scaling == "weak" else 0)
    if args.corpus == "planted":
        from oni_ml_amd.synth.corpus import planted_corpus
        c = planted_corpus(num_docs=args.docs, num_terms=args.vocab, num_topics=24, mean_tokens=25, tail=1.1,
                           max_tokens=300_000, seed=seed)
        names = [str(i) for i in range(c.num_terms)]
        info = {}
    elif args.corpus == "dns":
        from oni_ml_amd.pipeline.dns import synthetic_dns_corpus
        c, info, names = synthetic_dns_corpus(events=args.events, seed=seed, device=dev, return_names=True)
    else:
        from oni_ml_amd.pipeline.flow import synthetic_flow_corpus
        c, info, names = synthetic_flow_corpus(events=args.events, seed=seed, device=dev, return_names=True)
    if ctx.world_size > 1 and args.scaling == "weak":
        from oni_ml_amd.pipeline.flow import unify_vocabulary
        c, _ = unify_vocabulary(ctx, c, names)
    return c, info


def _settings(args):
    from oni_ml_amd.models.lda.settings import LDASettings
    st = LDASettings()
    st.gs_updates = int(args.gs_updates)
    return st


def _e2e(args, dev):
    """Wall-clock of the full pipeline (ml_ops.sh YYYYMMDD flow TOL equivalent) on a synthetic day."""
    import shutil
    import tempfile
    from oni_ml_amd import config as CFG
    from oni_ml_amd.pipeline import run
    from oni_ml_amd.synth.flow import generate_flow_day
    tmp = tempfile.mkdtemp(prefix="oni_e2e_")
    try:
        t0 = time.perf_counter()
        generate_flow_day(os.path.join(tmp, "in/"), events=args.events, seed=args.seed + 7)
        t_gen = time.perf_counter() - t0
        cfg = CFG.resolve("20160122", "flow", tol=args.e2e_tol, conf_path=None, environ={}, lpath=os.path.join(tmp, "ml"),
                          flow_path=os.path.join(tmp, "in"), backend=args.backend, topics=args.topics, verbose=False)
        _sync(dev)
        t0 = time.perf_counter()
        s = run(cfg, device=dev, log=lambda *a, **k: None)
        _sync(dev)
        wall = time.perf_counter() - t0
        return dict(e2e_wall_s=round(wall, 3), e2e_synth_input_s=round(t_gen, 3),
                    e2e_stage_s={k: round(v, 3) for k, v in s["stage_seconds"].items()},
                    e2e_em_iters=s["lda"]["em_iterations"], e2e_lda_timing=s["lda"].get("timing"), e2e_flagged=s.get("scored"), e2e_corpus=s.get("corpus"))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def _sync(dev):
    if torch.device(dev).type == "cuda":
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--gs-updates", type=int, default=0,
                    help="U, gamma refreshes per sweep of the fp64 engine (0: 32; > 32 needs K > 32; -1: the U "
                         "per K that meets lda-c parity, em.parity_gs_updates)")
    ap.add_argument("--events", type=int, default=None, help="events per GPU (default: flow 1M, dns 2M)")
    ap.add_argument("--corpus", choices=["flow", "dns", "planted"], default="flow",
                    help="flow: BASELINE headline (1-day netflow); dns: BASELINE config 4 (1-day DNS)")
    ap.add_argument("--docs", type=int, default=80_000)
    ap.add_argument("--vocab", type=int, default=8_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--streams", type=int, default=4, help="HIP streams for the E-step buckets")
    ap.add_argument("--batch", type=int, default=5,
                    help="EM iterations per host read-back (LDAEngine.run() batches LAG=5 when saving, 8 otherwise)")
    ap.add_argument("--converge", type=int, default=1, help="also time a full random-init run to convergence")
    ap.add_argument("--e2e", type=int, default=1, help="N=1: also time the whole ml_ops flow pipeline on the day")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"], help="cpu: gloo/torch rehearsal")
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32"],
                    help="fp64: lda-c arithmetic, block Gauss-Seidel (default); fp32: the experimental Jacobi mode")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: one day per GPU; strong: one day sharded over the GPUs")
    ap.add_argument("--e2e-tol", type=float, default=1e-5,
                    help="suspicion threshold of the timed e2e pipeline (1e-5 flags ~5 %% of the synthetic day)")
    args = ap.parse_args()
    args.backend = "hip" if args.device == "cuda" else "torch"
    if args.events is None:
        args.events = 2_000_000 if args.corpus == "dns" else 1_000_000

    from oni_ml_amd.parallel import dist as D
    ctx = D.init_from_env(expected_world=args.gpus, backend=None if args.device == "cuda" else "gloo")
    rank, world = ctx.rank, ctx.world_size
    dev = ctx.device if args.device == "cuda" else torch.device("cpu")

    from oni_ml_amd.models.lda.em import LDAEngine
    from oni_ml_amd.models.lda.settings import LDASettings

    t0 = time.perf_counter()
    corpus, info = build_corpus(args, rank, ctx, dev)
    t_corpus = time.perf_counter() - t0
    dist = ctx if world > 1 else None
    # weak scaling: each rank's corpus is its own document shard of the N-day corpus
    local = args.scaling == "weak"
    eng = LDAEngine(corpus, args.topics, _settings(args), backend=args.backend, device=dev, dist=dist, seed=args.seed,
                    local_shard=local, streams=args.streams, precision=args.precision)
    eng.init_random()
    docs_global = eng.global_docs

    def run_iters(n):
        # EM iterations exactly as LDAEngine.run() issues them without LAG saves: batches of --batch
        # iterations (one hipGraph replay each on one rank; E-step graph -> RCCL collectives -> M-step
        # graph on several), one batch always queued ahead of the host's read-back of the previous
        # batch's (likelihood, conv, alpha) history, the lda-c convergence test evaluated on the
        # device.  stop=False: every one of the n iterations runs in full (none is skipped by a
        # converged loop).
        batches = [min(args.batch, n - b) for b in range(0, n, args.batch)]
        recs = eng.em_iterations_pipelined(batches, True, docs_global, stop=False)
        assert len(recs) == n, (len(recs), n)

    run_iters(args.warmup)
    ctx.barrier()
    _sync(dev)
    t1 = time.perf_counter()
    run_iters(args.steps)
    _sync(dev)
    ctx.barrier()
    dt = time.perf_counter() - t1
    dt = ctx.allreduce_max(dt)
    ms = dt / args.steps * 1e3
    window_value = docs_global * args.steps / dt
    it = eng.iters.cpu().numpy()

    extra = dict(var_iter_mean=round(float(it.mean()), 3), var_iter_max=int(it.max()), var_max_iter=eng.var_max_iter)
    # variational iterations of the last E-step by document length (the long documents' share
    # of the E-step is words x iterations)
    lens = eng.corpus.lengths()
    by_len = {}
    for lo, hi in ((0, 16), (16, 64), (64, 256), (256, 1024), (1024, 4096), (4096, 1 << 40)):
        m = (lens > lo) & (lens <= hi)
        if m.any():
            by_len[f"{lo + 1}-{hi if hi < 1 << 40 else 'inf'}"] = [int(m.sum()), round(float(it[m].mean()), 2),
                                                                  int(it[m].max())]
    extra["var_iter_by_len"] = by_len
    value = window_value
    # the window's engine is done: its buffers go back to the allocator cache before the
    # to-convergence engine is built (one engine per process, as in a production run)
    eng_schedule, eng_xmode, eng_D, eng_nnz = eng.schedule, eng.exchange_mode, eng.D, eng.corpus.nnz
    del eng
    if args.converge:
        # to convergence: fresh engine and random init (seed + 1), lda-c's EM loop test on the device;
        # the clock includes the engine's construction (device CSR / CSC, length plans, buffers)
        ctx.barrier()
        _sync(dev)
        t2 = time.perf_counter()
        eng2 = LDAEngine(corpus, args.topics, _settings(args), backend=args.backend, device=dev, dist=dist,
                         seed=args.seed + 1, local_shard=local, precision=args.precision)
        _sync(dev)
        t_setup = time.perf_counter() - t2
        res = eng2.run()
        _sync(dev)
        tc = ctx.allreduce_max(time.perf_counter() - t2)
        t_setup = ctx.allreduce_max(t_setup)
        value = docs_global * res.em_iterations / tc
        extra.update(converge_seconds=round(tc, 4), converge_setup_seconds=round(t_setup, 4),
                     converge_em_iters=res.em_iterations, converge_docs_per_sec=round(value, 1),
                     converge_em_only_docs_per_sec=round(docs_global * res.em_iterations / max(tc - t_setup, 1e-9), 1),
                     final_likelihood=res.likelihoods[-1][0], final_alpha=res.alpha)
    if args.e2e and world == 1 and args.corpus == "flow" and args.events <= 2_000_000:
        extra.update(_e2e(args, dev))
    # the measured baseline is the 1-day netflow, K=20 corpus: other configs report no ratio
    base = _baseline() if (args.corpus == "flow" and args.topics == 20 and args.events == 1_000_000) else None
    if rank == 0:
        out = {
            "metric": METRIC if args.corpus != "dns" else "LDA docs/sec to convergence, 1-day DNS",
            "value": round(value, 1),
            "value_source": ("to convergence incl. engine setup: fresh engine + random init, lda-c EM loop test "
                             "(converge_* fields)"
                             if args.converge else "timed K-step window (no --converge run)"),
            "window_docs_per_sec": round(window_value, 1),
            "unit": "docs/s (docs x EM iterations / s, all ranks)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": (round(value / base, 2) if base else None),
            "dtype": ("fp64" if args.precision == "fp64" or args.backend != "hip" else
                      "fp32 E-step / fp64 likelihood, alpha, sufficient-statistic totals (reference lda-c: fp64)"),
            "schedule": eng_schedule,
            "precision_evidence": "profiles/r2_precision_parity.md",
            "data": (f"synthetic (1-day {'DNS' if args.corpus == 'dns' else 'netflow'} per GPU through the real "
                     "featurizer, random-init topics)" if args.corpus != "planted" else "synthetic planted-topic corpus"),
            "config": {
                "model": f"oni-lda-c variational EM LDA, K={args.topics}",
                "global_batch": docs_global,
                "seq_len": int(round(corpus.nnz / max(1, corpus.num_docs))),
                "precision": args.precision,
                "parallelism": f"dp{world}",
                "class_word_reduction": eng_xmode,
                "corpus": args.corpus,
                "events_per_gpu": args.events if args.corpus in ("flow", "dns") else None,
                "docs_per_gpu": eng_D,
                "vocab": corpus.num_terms,
                "nnz_per_gpu": eng_nnz,
                "max_doc_len": int(corpus.lengths().max()),
                "device": args.device,
            },
            "corpus_build_s": round(t_corpus, 3),
            **info,
            **extra,
        }
        print(json.dumps(out), flush=True)
    ctx.shutdown()


if __name__ == "__main__":
    main()
