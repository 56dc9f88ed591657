"""Row-sharded ``ml_ops`` pipeline: every stage runs on every rank (one process per GPU).

The reference runs featurization and scoring on ``SPK_EXEC`` Spark executors (ml_ops.sh:57,108),
LDA on 20 MPI ranks (:80) and lda_pre / lda_post serially.  Here each stage is split over the N ranks
and the ranks exchange only what the single-process pipeline would look at globally
(parallel/shardio.py):

  load       rank r ingests byte range r of FLOW_PATH (+ the feedback rows on the last rank)
  flow_pre   global cuts from merged histograms, global IP dictionary, local (ip, word) counts
  lda_pre    counts routed to the rank owning each document's id range; global word / document ids;
             entries moved to the nnz-balanced engine shards (corpus/sharded.py); words.dat,
             doc.dat, model.dat and doc_wc.dat written by all ranks at their byte offsets
  lda        the engine on this rank's shard; final.gamma = the ranks' blocks in rank order
  lda_post   doc_results.csv by document shard, word_results.csv by vocabulary slice
  flow_post  every rank scores its own rows; the survivors are merged into one ascending file

Every output file is byte-identical to the one-process pipeline's when the LDA model is
(ONI_DIST_DETERMINISTIC=chain, tests/test_sharded_pipeline.py).  Resumed runs (``--resume``) read
the finished stages' files on every rank.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..parallel import shardio as SIO
from . import common as C
from .runner import StageRunner


def _runner(cfg, ctx, device, log):
    return StageRunner(cfg.lpath, resume=cfg.resume, rank=ctx.rank, log=log,
                       sync=(torch.cuda.synchronize if device.type == "cuda" else None))


def write_corpus_files_sharded(ctx, lpath, sc, doc_names, word_names_of, threads=0):
    """words.dat (vocabulary slices), doc.dat and model.dat (document shards) from every rank."""
    from ..ops import native
    N, r = SIO.world(ctx), SIO.rank(ctx)
    L = native.lib()
    V = sc.word_keys.size
    v0, v1 = V * r // N, V * (r + 1) // N
    wn = word_names_of(sc.word_keys[v0:v1])
    t = L.format_rows(None, [("int", np.arange(v0, v1, dtype=np.int64)),
                             ("dict", wn, np.arange(v1 - v0, dtype=np.int32))], n=v1 - v0, threads=threads)
    SIO.write_segments(ctx, os.path.join(lpath, "words.dat"), [t])
    d0, d1 = sc.doc_range
    t = L.format_rows(None, [("int", np.arange(d0 + 1, d1 + 1, dtype=np.int64)),
                             ("dict", doc_names, np.arange(d1 - d0, dtype=np.int32))], n=d1 - d0, threads=threads)
    SIO.write_segments(ctx, os.path.join(lpath, "doc.dat"), [t])
    c = sc.corpus
    SIO.write_segments(ctx, os.path.join(lpath, "model.dat"),
                       [L.format_ldac_corpus(c.doc_ptr, c.word_idx, c.counts, threads=threads)])


def write_doc_wc_sharded(ctx, path, sc, ip_names, word_names_of, threads=0):
    """doc_wc.dat: this rank's block of every section, sections one after another."""
    from ..ops import native
    segs = []
    for sec in sc.lines:
        doc = sec.doc.cpu().numpy()
        ud, dinv = np.unique(doc, return_inverse=True)
        uw, winv = np.unique(sec.word.cpu().numpy(), return_inverse=True)
        segs.append(native.lib().format_rows(None, [("dict", ip_names.take(ud), dinv.astype(np.int32)),
                                                    ("dict", word_names_of(uw), winv.astype(np.int32)),
                                                    ("int", sec.count.cpu().numpy().astype(np.int64))],
                                             n=sec.n, threads=threads))
    SIO.write_segments(ctx, path, segs)


def _lda_stage(R, cfg, ctx, corpus, device, log, summary, local_shard, doc_offset=0):
    with R.stage("lda") as res:
        lres = C.run_lda(cfg, corpus, dist=ctx, device=device, log=log, local_shard=local_shard,
                         doc_offset=doc_offset)
        res["_defer"] = lres.close_files   # LAG / final model files: written while later stages run
        res.update(getattr(lres, "timing", {}))
        res.update(em_iterations=lres.em_iterations, likelihood=lres.likelihoods[-1][0] if lres.likelihoods else 0.0,
                   alpha=lres.alpha)
        m = lres.engine.metrics(lres.seconds, lres.em_iterations)
        res.update({k: v for k, v in m.items() if not isinstance(v, list)})
        R.emit(dict(stage="lda_detail", var_iter_hist=m["var_iter_hist"],
                    **{k: v for k, v in m.items() if not isinstance(v, list)}))
        summary["lda"] = dict(em_iterations=lres.em_iterations, timing=getattr(lres, "timing", {}), seconds=lres.seconds, alpha=lres.alpha,
                              likelihood=lres.likelihoods[-1][0] if lres.likelihoods else None)
    return lres


def _files_state(cfg, ctx):
    """Resume: the corpus files on every rank, this rank's shard of them (the engine's own rule,
    ``dist.engine_bounds``: the engine that re-runs the lda stage splits the documents the same way)."""
    from ..parallel.dist import engine_bounds
    corpus, doc_names, word_names = C.load_corpus_files(cfg.lpath)
    d0, d1 = engine_bounds(corpus.doc_ptr, ctx.world_size, cfg.topics)[ctx.rank]
    return corpus, doc_names, word_names, (d0, d1)


def run_flow(cfg, ctx, device=None, log=print) -> dict:
    from ..corpus.sharded import build_sharded
    from ..export import lda_post
    from ..features import flow as FF
    from ..features import flow_dist as FD
    from .flow import score_flow
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    R = _runner(cfg, ctx, device, log)
    summary = {}
    rank0 = ctx.rank == 0
    ft = sc = names = gmap = ws = None
    lres = None
    need_pre = not (R.done("lda_pre") and R.done("flow_pre"))
    if need_pre or not R.done("flow_post"):
        with R.stage("load") as res:
            ft = FD.load_flow_sharded(ctx, cfg.flow_path, cfg.feedback_path(), cfg.dupfactor, cfg.threads)
            res.update(rank_rows=ft.n)
            summary["input"] = dict(rows=ctx.allreduce_int(ft.n), feedback_rows=ctx.allreduce_int(ft.n_feedback))
    if need_pre:
        with R.stage("flow_pre") as res:
            sections, names, gmap, ws, cuts = FD.featurize_sharded(ctx, ft, device, cuts=cfg.fixed_cuts())
            if rank0:
                C.save_json(os.path.join(cfg.lpath, "flow_cuts.json"),
                            dict(cuts={k: v.tolist() for k, v in cuts.items()}, ports=ws.ports.tolist()))
            res["rank_pairs"] = sum(s.n for s in sections)
        with R.stage("lda_pre") as res:
            sc = build_sharded(ctx, sections, len(names), merge=not cfg.strict, device=device, K=cfg.topics)
            del sections
            doc_names = sc.doc_names = names.take(sc.doc_keys)
            write_corpus_files_sharded(ctx, cfg.lpath, sc, doc_names, ws.decode, cfg.threads)
            if cfg.write_doc_wc:
                write_doc_wc_sharded(ctx, os.path.join(cfg.lpath, "doc_wc.dat"), sc, names, ws.decode, cfg.threads)
            res.update(docs=sc.num_docs, terms=int(sc.word_keys.size), nnz=sc.nnz, rank_docs=sc.corpus.num_docs,
                       rank_nnz=sc.corpus.nnz)
            summary["corpus"] = dict(docs=sc.num_docs, terms=int(sc.word_keys.size), nnz=sc.nnz)
    else:
        R.skip("flow_pre")
        R.skip("lda_pre")
    try:
        tables, ip_rows = _lda_and_export(R, cfg, ctx, sc, names, gmap,
                                          (lambda k: ws.decode(k)) if ws is not None else None, device, log, summary)
        # ------------------------------------------------------------ flow_post
        if not R.done("flow_post"):
            with R.stage("flow_post") as res:
                res.update(score_flow(cfg, ft, tables, device, log if rank0 else (lambda *a, **k: None),
                                      ctx=ctx, ip_rows=ip_rows))
                summary["scored"] = res.get("flagged")
        else:
            R.skip("flow_post")
    except BaseException:
        R.finish_deferred(suppress=True)
        raise
    R.finish_deferred()
    summary["stage_seconds"] = dict(R.times)
    return summary


def run_dns(cfg, ctx, device=None, log=print) -> dict:
    from ..corpus.sharded import build_sharded
    from ..export import lda_post
    from ..features import dns as FD
    from ..features import dns_dist as FDD
    from .dns import score_dns
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    R = _runner(cfg, ctx, device, log)
    summary = {}
    rank0 = ctx.rank == 0
    tab = sc = names = gmap = wsp = top = None
    need_pre = not (R.done("lda_pre") and R.done("dns_pre"))
    if need_pre or not R.done("dns_post"):
        with R.stage("load") as res:
            tab = FDD.load_dns_sharded(ctx, cfg.dns_path, cfg.feedback_path(), cfg.dupfactor, strict=cfg.strict)
            top = FD.load_top_domains(cfg.top1m)
            if not top and rank0:
                log(f"warning: top-1m list {cfg.top1m!r} not found; every domain gets top_domain 0/2")
            res.update(rank_rows=tab.n, top_domains=len(top))
            summary["input"] = dict(rows=ctx.allreduce_int(tab.n), feedback_rows=ctx.allreduce_int(tab.n_feedback),
                                    dropped=ctx.allreduce_int(tab.dropped))
    if need_pre:
        with R.stage("dns_pre") as res:
            sections, names, gmap, wsp, cuts = FDD.featurize_sharded(ctx, tab, device, top, threads=cfg.threads)
            if rank0:
                C.save_json(os.path.join(cfg.lpath, "dns_cuts.json"), dict(cuts={k: v.tolist() for k, v in cuts.items()}))
            res["rank_pairs"] = sum(s.n for s in sections)
        with R.stage("lda_pre") as res:
            sc = build_sharded(ctx, sections, len(names), device=device, K=cfg.topics)
            del sections
            doc_names = sc.doc_names = names.take(sc.doc_keys)
            write_corpus_files_sharded(ctx, cfg.lpath, sc, doc_names, wsp.decode, cfg.threads)
            if cfg.write_doc_wc:
                write_doc_wc_sharded(ctx, os.path.join(cfg.lpath, "doc_wc.dat"), sc, names, wsp.decode, cfg.threads)
            res.update(docs=sc.num_docs, terms=int(sc.word_keys.size), nnz=sc.nnz, rank_docs=sc.corpus.num_docs,
                       rank_nnz=sc.corpus.nnz)
            summary["corpus"] = dict(docs=sc.num_docs, terms=int(sc.word_keys.size), nnz=sc.nnz)
    else:
        R.skip("dns_pre")
        R.skip("lda_pre")
    try:
        tables, ip_rows = _lda_and_export(R, cfg, ctx, sc, names, gmap,
                                          (lambda k: wsp.decode(k)) if wsp is not None else None, device, log, summary)
        if not R.done("dns_post"):
            with R.stage("dns_post") as res:
                res.update(score_dns(cfg, tab, top, tables, device, log if rank0 else (lambda *a, **k: None),
                                     ctx=ctx, ip_map=ip_rows))
                summary["scored"] = res.get("flagged")
        else:
            R.skip("dns_post")
    except BaseException:
        R.finish_deferred(suppress=True)
        raise
    R.finish_deferred()
    summary["stage_seconds"] = dict(R.times)
    return summary


def _lda_and_export(R, cfg, ctx, sc, names, gmap, decode, device, log, summary):
    """lda + lda_post of the sharded pipeline (in memory after a fresh pre stage, from the files on
    resume).  Returns (scoring tables, doc row of every local ip id or None)."""
    from ..export import lda_post
    word_names = doc_names = None
    if sc is not None:
        doc_names = getattr(sc, "doc_names", None)
        if doc_names is None:
            doc_names = names.take(sc.doc_keys)
    gamma = log_beta = None
    if not R.done("lda"):
        if sc is not None:
            lres = _lda_stage(R, cfg, ctx, sc.corpus, device, log, summary, True, sc.doc_range[0])
        else:
            corpus, all_docs, word_names, (d0, d1) = _files_state(cfg, ctx)
            doc_names = all_docs[d0:d1]
            lres = _lda_stage(R, cfg, ctx, corpus, device, log, summary, False)
        gamma, log_beta = lres.gamma, lres.log_beta
    else:
        R.skip("lda")
    ip_rows = None
    if not R.done("lda_post"):
        if gamma is None:
            from ..models.lda.estimate import load_final_rows
            corpus, all_docs, _, (d0, d1) = _files_state(cfg, ctx)
            doc_names = all_docs[d0:d1]
            gamma, log_beta = load_final_rows(cfg.lpath, d0, d1)
        with R.stage("lda_post"):
            if sc is not None:
                # nothing replicated: this rank's θ rows and vocabulary slice, the word map hash-partitioned,
                # the doc row of an ip id in id-range slices (shardio.range_put / fetch_rows)
                V = int(log_beta.shape[1])
                N, r = SIO.world(ctx), SIO.rank(ctx)
                v0, v1 = V * r // N, V * (r + 1) // N
                if word_names is None:
                    word_names = decode(sc.word_keys[v0:v1])
                elif len(word_names) == V:
                    word_names = word_names[v0:v1]
                th, ph, wn = lda_post.export_sharded(ctx, doc_names, gamma, word_names, log_beta,
                                                     os.path.join(cfg.lpath, "doc_results.csv"),
                                                     os.path.join(cfg.lpath, "word_results.csv"),
                                                     strict=cfg.strict, read_back=True, gather=False, num_words=V)
                ws = SIO.range_starts(V, N)
                tables = C.ShardedTables(ctx, th, list(sc.bounds), ph, ws, SIO.DistDict(ctx, wn, np.arange(v0, v1)))
                d0, d1 = sc.doc_range
                ip_doc = SIO.range_put(ctx, sc.doc_keys, np.arange(d0, d1, dtype=np.int64), len(names), fill=-1)
                ip_rows = SIO.fetch_rows(ctx, ip_doc, SIO.range_starts(len(names), N), gmap)
            else:
                if word_names is None:
                    word_names = C.load_corpus_files(cfg.lpath)[2]
                th, ph, wn = lda_post.export_sharded(ctx, doc_names, gamma, word_names, log_beta,
                                                     os.path.join(cfg.lpath, "doc_results.csv"),
                                                     os.path.join(cfg.lpath, "word_results.csv"),
                                                     strict=cfg.strict, read_back=True)
                tables = C.ModelTables(C.load_corpus_files(cfg.lpath)[1], th, wn, ph)
    else:
        R.skip("lda_post")
        tables = C.load_model_tables(cfg.lpath)
    return tables, ip_rows
