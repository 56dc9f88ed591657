"""Netflow suspicious-connects pipeline (ml_ops.sh YYYYMMDD flow [TOL]).

Stages (reference call stack SURVEY.md §3.1):
  flow_pre   featurize FLOW_PATH (+ analyst feedback x DUPFACTOR) -> (ip, word) counts   [flow_pre_lda.scala]
  lda_pre    words.dat / doc.dat / model.dat (+ doc_wc.dat)                               [lda_pre.py]
  lda        variational EM on the GPU(s) -> final.{beta,gamma,other}, likelihood.dat    [oni-lda-c]
  lda_post   doc_results.csv / word_results.csv                                          [lda_post.py]
  flow_post  re-featurize raw rows, score, filter < TOL, sort -> flow_results.csv        [flow_post_lda.scala]

Everything between stages stays in memory (device tensors / host arrays); the
text files are written as the compatibility contract and are what `--resume`
reloads when earlier stages are already complete.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from ..corpus.builder import concat, count_pairs, lda_pre
from ..features import flow as FF
from ..ops import sortgroup as SG
from ..score import scorer as S
from . import common as C
from . import prefetch
from .runner import StageRunner


def _host_cuts(ft, which: str):
    """flow_pre's ("all") or flow_post's ("raw") cuts computed by the input prefetch (pipeline/prefetch.py
    load_flow_inputs), or None."""
    hc = getattr(ft, "host_cuts", None) if ft is not None else None
    return hc.get(which) if hc else None


def _word_names(ws: FF.FlowWordSpace, keys: np.ndarray):
    return ws.decode(keys)


def run(cfg, dist=None, device=None, log=print) -> dict:
    if dist is not None and dist.active:
        from .sharded import run_flow
        return run_flow(cfg, dist, device, log)
    rank = 0 if dist is None else dist.rank
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    R = StageRunner(cfg.lpath, resume=cfg.resume, rank=rank, log=log,
                    sync=(torch.cuda.synchronize if device.type == "cuda" else None))
    summary = {}
    ft = feat = ws = built = None
    doc_names = word_names = None

    # ------------------------------------------------------------------ pre
    need_pre = not (R.done("lda_pre") and R.done("flow_pre"))
    sharded = False     # several ranks: pipeline/sharded.py
    if rank == 0 and (need_pre or not R.done("flow_post")) and not sharded:
        with R.stage("load") as res:
            ft = prefetch.take(prefetch.flow_key(cfg))
            res["prefetched"] = ft is not None
            if ft is None:
                ft = FF.load_flow(cfg.flow_path, cfg.feedback_path(), cfg.dupfactor, cfg.threads)
            res.update(ft.stats())
            summary["input"] = ft.stats()
    if need_pre:
        if rank == 0:
            with R.stage("flow_pre") as res:
                # cuts: CUT, else those the input prefetch computed on the host, else the device ECDF
                cuts = cfg.fixed_cuts()
                feat = FF.featurize(ft, device, cuts=cuts if cuts is not None else _host_cuts(ft, "all"))
                ws = FF.word_space_for(feat)
                src, dst = FF.word_keys(feat, ws)
                dwc = concat([count_pairs(feat.sip, src, feat.weight), count_pairs(feat.dip, dst, feat.weight)],
                             merge=not cfg.strict)
                C.save_json(os.path.join(cfg.lpath, "flow_cuts.json"),
                            dict(cuts={k: v.tolist() for k, v in feat.cuts.items()}, ports=ws.ports.tolist()))
                res["pairs"] = dwc.n
                log(f"cuts: time={feat.cuts['time'].tolist()} ibyt={feat.cuts['ibyt'].tolist()} "
                    f"ipkt={feat.cuts['ipkt'].tolist()}")
            with R.stage("lda_pre") as res:
                built = lda_pre(dwc)
                ipn = ft.ip_names
                doc_names = [ipn[i] for i in built.doc_keys.tolist()]
                word_names = _word_names(ws, built.word_keys)
                lp, b_, dn_, wn_ = cfg.lpath, built, doc_names, word_names

                # host copies here, not on the writer thread (DocWordCounts.to_host)
                dwc_h = dwc.to_host() if cfg.write_doc_wc else None

                def write_files():
                    if dwc_h is not None:
                        from ..corpus.builder import write_doc_wc
                        write_doc_wc(os.path.join(lp, "doc_wc.dat"), dwc_h, ipn, C.vocab_lookup(b_.word_keys, wn_))
                    C.write_corpus_files(lp, b_, dn_, wn_)
                # the text files are the stage contract, not an input of the in-memory lda stage: written
                # on a thread while the GPU runs EM; the lda_pre marker waits for them (finish_deferred)
                if True:   # text files on a thread beside the EM (profiles/r3_tuning_log.md: e2e 0.66 -> 0.53 s)
                    res["_defer"] = C.background(write_files, "oni-lda-pre-writer")
                else:
                    write_files()
                res.update(docs=built.corpus.num_docs, terms=built.corpus.num_terms, nnz=built.corpus.nnz)
                summary["corpus"] = dict(docs=built.corpus.num_docs, terms=built.corpus.num_terms, nnz=built.corpus.nnz)
    elif not sharded:
        R.skip("flow_pre")
        R.skip("lda_pre")

    # ------------------------------------------------------------------ lda
    corpus = built.corpus if built is not None else None
    if not R.done("lda"):
        if corpus is None and rank == 0:
            corpus, doc_names, word_names = C.load_corpus_files(cfg.lpath)
        if dist is not None and dist.world_size > 1 and not sharded:
            corpus = dist.broadcast_corpus(corpus)
        with R.stage("lda") as res:
            lres = C.run_lda(cfg, corpus, dist=dist, device=device, log=log)
            res["_defer"] = lres.close_files   # LAG / final model files: written while later stages run
            res.update(getattr(lres, "timing", {}))
            res.update(em_iterations=lres.em_iterations, likelihood=lres.likelihoods[-1][0] if lres.likelihoods else 0.0,
                       alpha=lres.alpha)
            m = lres.engine.metrics(lres.seconds, lres.em_iterations)
            res.update({k: v for k, v in m.items() if not isinstance(v, list)})
            R.emit(dict(stage="lda_detail", var_iter_hist=m["var_iter_hist"], **{k: v for k, v in m.items()
                                                                                   if not isinstance(v, list)}))
            summary["lda"] = dict(em_iterations=lres.em_iterations, timing=getattr(lres, "timing", {}), seconds=lres.seconds, alpha=lres.alpha,
                                  likelihood=lres.likelihoods[-1][0] if lres.likelihoods else None)
        gamma, log_beta = lres.gamma, lres.log_beta
    else:
        R.skip("lda")
        gamma = log_beta = None
    if rank != 0:
        R.finish_deferred()
        return summary
    try:

        # ------------------------------------------------------------- lda_post
        if not R.done("lda_post"):
            if doc_names is None:
                _, doc_names, word_names = C.load_corpus_files(cfg.lpath)
            if gamma is None:
                from ..models.lda.estimate import load_final
                gamma, log_beta = load_final(cfg.lpath)
            with R.stage("lda_post") as res:
                # deferred text: measured no e2e gain on the 1-day tables (tuning log); on from
                # DEFER_POST_VALUES (2^26) values, where formatting ~1 G values (config 5) overlaps scoring
                big = (len(doc_names) + len(word_names)) * int(gamma.shape[1]) >= C.DEFER_POST_VALUES
                if big:
                    # the result files are written on a thread while flow_post scores (its tables
                    # are the text round trip of the same values); the lda_post marker waits for them
                    from ..export import lda_post as LP
                    th, ph, wn, join = LP.export_deferred(doc_names, gamma, word_names, log_beta,
                                                          os.path.join(cfg.lpath, "doc_results.csv"),
                                                          os.path.join(cfg.lpath, "word_results.csv"),
                                                          strict=cfg.strict)
                    tables = C.ModelTables(list(doc_names), th, wn, ph)
                    res["_defer"] = join
                else:
                    tables = C.run_export(cfg, doc_names, gamma, word_names, log_beta, read_back=True)
                if built is not None and ws is not None and not cfg.strict:
                    tables.word_keys, tables.key_space = np.asarray(built.word_keys), ws
        else:
            R.skip("lda_post")
            tables = C.load_model_tables(cfg.lpath)

        # ------------------------------------------------------------ flow_post
        if not R.done("flow_post"):
            if ft is None:
                # row-sharded pre stages: rank 0 reads the whole day for the scoring pass
                ft = prefetch.take(prefetch.flow_key(cfg)) or FF.load_flow(cfg.flow_path, cfg.feedback_path(),
                                                                          cfg.dupfactor, cfg.threads)
            # documents built in this process: ip dictionary id -> doc row without the name lookup
            ip_rows = C.doc_rows_of(built.doc_keys, len(ft.ip_names)) if built is not None else None
            with R.stage("flow_post") as res:
                res.update(score_flow(cfg, ft, tables, device, log, ip_rows=ip_rows))
                summary["scored"] = res.get("flagged")
        else:
            R.skip("flow_post")
    except BaseException:
        R.finish_deferred(suppress=True)
        raise
    R.finish_deferred()
    summary["stage_seconds"] = dict(R.times)
    return summary


def score_flow(cfg, ft: FF.FlowTable, tables: C.ModelTables, device, log=print, ctx=None, ip_rows=None) -> dict:
    """flow_post_lda.scala: features of raw rows, θ·φ per side, min, < TOL, ascending, 37-column rows.

    ``ctx`` (several ranks): ``ft`` holds this rank's rows; the cuts come from every rank's raw rows,
    and the survivors of all ranks are merged into one ascending file (``shardio.merge_sorted_rows``,
    the sortByKey shuffle).  ``ip_rows``: doc row of every ip dictionary id of ``ft`` (-1: not a
    document) -- replaces the name lookup through ``tables.doc_index()``."""
    from ..parallel import shardio as SIO
    multi = ctx is not None and ctx.active
    cuts = cfg.fixed_cuts()          # fixed CUT cuts apply to both stages (flow_pre_lda.scala:95-98)
    if cuts is None and not cfg.strict:
        saved = C.load_json(os.path.join(cfg.lpath, "flow_cuts.json"))
        cuts = {k: np.asarray(v, np.float64) for k, v in saved["cuts"].items()}
    if cuts is None and multi:
        # flow_post_lda.scala:143-150: the cuts of the raw rows (no feedback) of the whole day
        from ..features import flow_dist as FDS
        cols, w = FDS.table_columns(ft, ft.n_raw, torch.device(device))
        cuts = {k: v.cpu().numpy() for k, v in FDS.global_cuts(ctx, cols, w, device).items()}
    if cuts is None and not multi:
        cuts = _host_cuts(ft, "raw")
    feat = FF.featurize(ft, device, cuts=cuts, raw_only=True)
    # keys straight to φ rows when the tables carry this process's vocabulary (compat=fixed: names are
    # untruncated and unique, so key -> name -> row is key -> row; the cuts are the pre stage's, so the
    # pre stage's key space encodes these events too); otherwise through the names as written (strict:
    # 20-byte keys never match long words, later duplicate rows win)
    fast = (not multi and not cfg.strict and getattr(tables, "word_keys", None) is not None
            and getattr(tables, "key_space", None) is not None)
    ws = tables.key_space if fast else FF.word_space_for(feat)
    src, dst = FF.word_keys(feat, ws)
    both = torch.cat([src, dst])
    uk, inv = SG.unique(both, return_inverse=True)
    uk_np = uk.cpu().numpy()
    if fast:
        wk = np.asarray(tables.word_keys, np.int64)
        o = np.argsort(wk, kind="stable")
        pos = np.minimum(np.searchsorted(wk[o], uk_np), max(wk.size - 1, 0))
        word_rows = np.where(wk[o][pos] == uk_np, o[pos], -1) if wk.size else np.full(uk_np.size, -1, np.int64)
        unames = None
    else:
        unames = ws.decode(uk_np)
        word_rows = tables.word_rows(unames)
    ipn = ft.ip_names
    if ip_rows is None:
        ip_rows = np.fromiter((tables.doc_index().get(n, -1) for n in ipn), dtype=np.int64, count=len(ipn))
    # the rows these events reference: the whole tables (one process) or fetched from their ranks
    th, ph, drow, wrow = tables.compact(ip_rows, word_rows)
    widx = SG.gather(torch.from_numpy(wrow).to(device), inv)
    w_src, w_dst = widx[: src.numel()], widx[src.numel():]
    didx = torch.from_numpy(drow).to(device)
    K = tables.K
    if cfg.strict and K != 20:
        raise ValueError("compat=strict scores over exactly 20 topics (flow_post_lda.scala:232)")
    model = S.TopicModel.build(th, ph, S.default_value("flow", K, cfg.strict), device)
    sa, sb, key, flag = S.score(model, SG.gather(didx, feat.sip), w_src, SG.gather(didx, feat.dip), w_dst, cfg.tol)
    qs = S.key_quantiles(key)
    order = S.rank_flagged(key, flag)
    n = int(order.size)
    out = os.path.join(cfg.lpath, "flow_results.csv")
    # output columns: 27 raw + time + ibyt_bin + ipkt_bin + time_bin + word_port + ip_pair + src/dest word + scores
    o_t = torch.from_numpy(order).to(device)
    inv_src = SG.gather(inv[: src.numel()], o_t).cpu().numpy().astype(np.int32)
    inv_dst = SG.gather(inv[src.numel():], o_t).cpu().numpy().astype(np.int32)
    if unames is None:      # names only for the words of the flagged rows
        need = np.unique(np.concatenate([inv_src, inv_dst]))
        unames = ws.decode(uk_np[need])
        inv_src = np.searchsorted(need, inv_src).astype(np.int32)
        inv_dst = np.searchsorted(need, inv_dst).astype(np.int32)
    sel = lambda t: SG.gather(t, o_t).cpu().numpy()
    cols = [
        ("table", ft.table, order),
        ("java", sel(feat.time)),
        ("int", sel(feat.ibyt_bin).astype(np.int64)),
        ("int", sel(feat.ipkt_bin).astype(np.int64)),
        ("int", sel(feat.time_bin).astype(np.int64)),
        ("java", sel(feat.word_port)),
        ("pair", ipn, sel(feat.sip).astype(np.int32), sel(feat.dip).astype(np.int32)),
        ("dict", unames, inv_src),
        ("dict", unames, inv_dst),
        ("java", sel(sa)),
        ("java", sel(sb)),
    ]
    from ..ops import native
    if multi:
        text, ends = native.lib().format_rows(None, cols, n=n, row_ends=True, threads=cfg.threads)
        total = SIO.merge_sorted_rows(ctx, sel(key).astype(np.float64), text, ends, out)
        log(f"flow_post: {total} events with score < {cfg.tol} written to {out} ({n} from rank {ctx.rank})")
        return dict(flagged=total, rank_flagged=n, events=ctx.allreduce_int(int(feat.time.numel())), **qs)
    native.lib().write_rows(out, None, cols, threads=cfg.threads, n=n)
    log(f"flow_post: {n} events with score < {cfg.tol} written to {out}")
    return dict(flagged=n, events=int(feat.time.numel()), **qs)


def synthetic_flow_corpus(events: int = 1_000_000, seed: int = 0, workdir: Optional[str] = None, device=None,
                          strict: bool = True, threads: int = 8, return_names: bool = False, chunk_events: int = 0):
    """Synthetic netflow day -> featurized -> lda-c corpus (the bench / test input path).
    ``chunk_events``: generate part file by part file (a month: one file per day, synth/flow.py).

    Returns (Corpus, info dict with stage timings[, word names])."""
    import tempfile
    import time
    from ..synth.flow import generate_flow_day
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    tmp = tempfile.mkdtemp(prefix="oni_flow_") if workdir is None else workdir
    t0 = time.perf_counter()
    gen = generate_flow_day(os.path.join(tmp, "in/"), events=events, seed=seed, threads=threads,
                            chunk_events=chunk_events)
    t1 = time.perf_counter()
    ft = FF.load_flow(os.path.join(tmp, "in"), None, 1000, threads)
    t2 = time.perf_counter()
    feat = FF.featurize(ft, device)
    ws = FF.word_space_for(feat)
    src, dst = FF.word_keys(feat, ws)
    dwc = concat([count_pairs(feat.sip, src, feat.weight), count_pairs(feat.dip, dst, feat.weight)], merge=not strict)
    built = lda_pre(dwc)
    if device.type == "cuda":
        torch.cuda.synchronize()
    t3 = time.perf_counter()
    if workdir is None:
        import shutil
        shutil.rmtree(tmp, ignore_errors=True)
    info = dict(events=events, synth_s=round(t1 - t0, 3), ingest_s=round(t2 - t1, 3), featurize_corpus_s=round(t3 - t2, 3))
    if return_names:
        return built.corpus, info, ws.decode(built.word_keys)
    return built.corpus, info


def unify_vocabulary(ctx, corpus, word_names):
    """Map a rank-local corpus onto the union vocabulary of all ranks (sorted word strings).

    Data-parallel EM all-reduces class_word [V, K]: every rank must index the
    same words the same way.  Ranks that featurize different days (weak-scaling
    bench, multi-day runs) see different word sets; their union, ordered by the
    word string, is the shared dictionary."""
    from ..corpus.csr import Corpus
    names = list(word_names)
    if ctx is not None and ctx.initialized:
        import torch.distributed as td
        gathered = [None] * ctx.world_size
        td.all_gather_object(gathered, names)
    else:
        gathered = [names]
    vocab = sorted(set().union(*[set(g) for g in gathered]))
    index = {w: i for i, w in enumerate(vocab)}
    remap = np.fromiter((index[w] for w in names), dtype=np.int32, count=len(names))
    c = Corpus(corpus.doc_ptr, remap[corpus.word_idx], corpus.counts, len(vocab), meta=dict(corpus.meta))
    return c, vocab
