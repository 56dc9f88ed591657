"""DNS suspicious-connects pipeline (ml_ops.sh YYYYMMDD dns [TOL]).

Stages: load -> dns_pre -> lda_pre -> lda -> lda_post -> dns_post
(reference: dns_pre_lda.scala, lda_pre.py, oni-lda-c, lda_post.py,
dns_post_lda.scala).  Output dns_results.csv has 16
columns: the 8 input fields, domain, subdomain, subdomain.length,
num.periods, subdomain.entropy, top_domain, word, score (dns_post_lda.scala:326-331).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..corpus.builder import count_pairs, lda_pre
from ..features import dns as FD
from ..score import scorer as S
from . import common as C
from . import prefetch
from .runner import StageRunner


def run(cfg, dist=None, device=None, log=print) -> dict:
    if dist is not None and dist.active:
        from .sharded import run_dns
        return run_dns(cfg, dist, device, log)
    rank = 0 if dist is None else dist.rank
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    R = StageRunner(cfg.lpath, resume=cfg.resume, rank=rank, log=log,
                    sync=(torch.cuda.synchronize if device.type == "cuda" else None))
    summary = {}
    tab = built = None
    doc_names = word_names = None
    top = None
    pre_host = None      # dns_pre's name features: dns_post takes its raw rows' slice
    need_pre = not (R.done("lda_pre") and R.done("dns_pre"))
    if rank == 0 and (need_pre or not R.done("dns_post")):
        with R.stage("load") as res:
            got = prefetch.take(prefetch.dns_key(cfg))
            res["prefetched"] = got is not None
            if got is not None:
                tab, top, pre_host = got
            else:
                tab = FD.load_dns(cfg.dns_path, cfg.feedback_path(), cfg.dupfactor, strict=cfg.strict)
                top = FD.load_top_domains(cfg.top1m)
            if not top:
                log(f"warning: top-1m list {cfg.top1m!r} not found; every domain gets top_domain 0/2")
            res.update(rows=tab.n, raw_rows=tab.n_raw, feedback_rows=tab.n_feedback, dropped=tab.dropped,
                       top_domains=len(top))
            summary["input"] = dict(rows=tab.n, feedback_rows=tab.n_feedback, dropped=tab.dropped)
    if need_pre:
        if rank == 0:
            with R.stage("dns_pre") as res:
                feat = FD.featurize(tab, device, top, threads=cfg.threads, host=pre_host)
                pre_host = feat.host
                wsp = FD.DnsWordSpace(feat.cuts, feat.qpairs)
                dwc = count_pairs(feat.ip, feat.word_key, feat.weight)
                C.save_json(os.path.join(cfg.lpath, "dns_cuts.json"), dict(cuts={k: v.tolist() for k, v in feat.cuts.items()}))
                res["pairs"] = dwc.n
                log("cuts: " + " ".join(f"{k}={v.tolist()}" for k, v in feat.cuts.items()))
            with R.stage("lda_pre") as res:
                built = lda_pre(dwc)
                doc_names = [feat.ip_names[i] for i in built.doc_keys.tolist()]
                word_names = wsp.decode(built.word_keys)
                lp, b_, dn_, wn_, ipn = cfg.lpath, built, doc_names, word_names, feat.ip_names

                # host copies here, not on the writer thread (DocWordCounts.to_host)
                dwc_h = dwc.to_host() if cfg.write_doc_wc else None

                def write_files():
                    if dwc_h is not None:
                        from ..corpus.builder import write_doc_wc
                        write_doc_wc(os.path.join(lp, "doc_wc.dat"), dwc_h, ipn, C.vocab_lookup(b_.word_keys, wn_))
                    C.write_corpus_files(lp, b_, dn_, wn_)
                # as in the flow pipeline: the text files on a thread during EM, the marker waits for them
                if True:   # text files on a thread beside the EM (pipeline/flow.py)
                    res["_defer"] = C.background(write_files, "oni-lda-pre-writer")
                else:
                    write_files()
                res.update(docs=built.corpus.num_docs, terms=built.corpus.num_terms, nnz=built.corpus.nnz)
                summary["corpus"] = dict(docs=built.corpus.num_docs, terms=built.corpus.num_terms, nnz=built.corpus.nnz)
    else:
        R.skip("dns_pre")
        R.skip("lda_pre")

    corpus = built.corpus if built is not None else None
    if not R.done("lda"):
        if corpus is None and rank == 0:
            corpus, doc_names, word_names = C.load_corpus_files(cfg.lpath)
        if dist is not None and dist.world_size > 1:
            corpus = dist.broadcast_corpus(corpus)
        with R.stage("lda") as res:
            lres = C.run_lda(cfg, corpus, dist=dist, device=device, log=log)
            res["_defer"] = lres.close_files   # LAG / final model files: written while later stages run
            res.update(getattr(lres, "timing", {}))
            res.update(em_iterations=lres.em_iterations, alpha=lres.alpha)
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

        if not R.done("lda_post"):
            if doc_names is None:
                _, doc_names, word_names = C.load_corpus_files(cfg.lpath)
            if gamma is None:
                from ..models.lda.estimate import load_final
                gamma, log_beta = load_final(cfg.lpath)
            with R.stage("lda_post"):
                tables = C.run_export(cfg, doc_names, gamma, word_names, log_beta, read_back=True)
        else:
            R.skip("lda_post")
            tables = C.load_model_tables(cfg.lpath)

        if not R.done("dns_post"):
            with R.stage("dns_post") as res:
                res.update(score_dns(cfg, tab, top, tables, device, log, host=pre_host))
                summary["scored"] = res.get("flagged")
        else:
            R.skip("dns_post")
    except BaseException:
        R.finish_deferred(suppress=True)
        raise
    R.finish_deferred()
    summary["stage_seconds"] = dict(R.times)
    return summary


def score_dns(cfg, tab: FD.DnsTable, top, tables: C.ModelTables, device, log=print, ctx=None, ip_map=None,
              host=None) -> dict:
    """dns_post_lda.scala:108-331.  ``ctx`` (several ranks): ``tab`` holds this rank's rows; cuts over
    every rank's raw rows; the survivors of all ranks merged into one ascending file.  ``ip_map``:
    doc row of every ip_dst id of the pre-LDA dictionary of ``tab`` (its raw rows' ids are a prefix)."""
    from ..parallel import shardio as SIO
    multi = ctx is not None and ctx.active
    cuts = None
    if not cfg.strict:
        cuts = {k: np.asarray(v, np.float64) for k, v in C.load_json(os.path.join(cfg.lpath, "dns_cuts.json"))["cuts"].items()}
    elif multi:
        from ..features import dns_dist as FDD
        cuts = FDD.global_cuts(ctx, tab, top, device, raw_only=True, threads=cfg.threads)
    feat = FD.featurize(tab, device, top, cuts=cuts, raw_only=True, threads=cfg.threads, host=host)
    wsp = FD.DnsWordSpace(feat.cuts, feat.qpairs)
    from ..ops import sortgroup as SG
    uk, inv = SG.unique(feat.word_key, return_inverse=True)
    unames = wsp.decode(uk.cpu().numpy())
    if ip_map is not None:
        m = np.asarray(ip_map, np.int64)[:len(feat.ip_names)]
    else:
        di = tables.doc_index()
        m = np.fromiter((di.get(n, -1) for n in feat.ip_names), dtype=np.int64, count=len(feat.ip_names))
    # the rows these queries reference: the whole tables (one process) or fetched from their ranks
    th, ph, drow, wrow = tables.compact(m, tables.word_rows(unames))
    widx = SG.gather(torch.from_numpy(wrow).to(device), inv)
    didx = SG.gather(torch.from_numpy(drow).to(device), feat.ip)
    K = tables.K
    if cfg.strict and K != 20:
        raise ValueError("compat=strict scores over exactly 20 topics (dns_post_lda.scala:316)")
    model = S.TopicModel.build(th, ph, S.default_value("dns", K, cfg.strict), device)
    sc, _, key, flag = S.score(model, didx, widx, None, None, cfg.tol)
    order = S.rank_flagged(key, flag)
    n = int(order.size)
    out = os.path.join(cfg.lpath, "dns_results.csv")
    # the flagged rows' 8 input columns, dictionary-encoded by Arrow on a thread each (its kernels
    # release the GIL)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(FD.COLUMNS)) as ex:
        enc = list(ex.map(lambda c: tab.take_encoded(c, order), FD.COLUMNS))
    cols = [("dict", names, ids) for ids, names in enc]
    H = feat.host
    o_t = torch.from_numpy(order).to(sc.device)
    cols += [
        ("dict", H["domains"], H["domain_id"][order]),
        ("dict", H["subdomains"], H["subdomain_id"][order]),
        ("int", H["subdomain_length"][order].astype(np.int64)),
        ("int", H["num_periods"][order].astype(np.int64)),
        ("java", H["entropy"][order]),
        ("int", H["top_domain"][order].astype(np.int64)),
        ("dict", unames, inv[torch.from_numpy(order).to(inv.device)].cpu().numpy().astype(np.int32)),
        ("java", sc[o_t].cpu().numpy()),
    ]
    from ..ops import native
    if multi:
        text, ends = native.lib().format_rows(None, cols, n=n, row_ends=True, threads=cfg.threads)
        total = SIO.merge_sorted_rows(ctx, key[o_t].cpu().numpy().astype(np.float64), text, ends, out)
        log(f"dns_post: {total} queries with score < {cfg.tol} written to {out} ({n} from rank {ctx.rank})")
        return dict(flagged=total, rank_flagged=n, events=ctx.allreduce_int(int(feat.word_key.numel())))
    native.lib().write_rows(out, None, cols, threads=cfg.threads, n=n)
    log(f"dns_post: {n} queries with score < {cfg.tol} written to {out}")
    return dict(flagged=n, events=int(feat.word_key.numel()))


def synthetic_dns_corpus(events: int = 2_000_000, seed: int = 0, device=None, strict: bool = True, threads: int = 8,
                         return_names: bool = False, n_names: int = None, n_clients: int = None):
    """Synthetic DNS day -> featurized (dns_pre_lda semantics) -> lda-c corpus: the bench / test input path.

    Name and client populations grow with the day's size (a 2M-query day: 200k names, 50k clients)."""
    import shutil
    import tempfile
    import time
    from ..synth.dns import generate_dns_day
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    n_names = n_names or max(20_000, events // 10)
    n_clients = n_clients or max(5_000, events // 40)
    tmp = tempfile.mkdtemp(prefix="oni_dns_")
    try:
        t0 = time.perf_counter()
        gen = generate_dns_day(os.path.join(tmp, "in/"), events=events, seed=seed, n_names=n_names,
                               n_clients=n_clients, with_edge_rows=False)
        t1 = time.perf_counter()
        tab = FD.load_dns(gen["dns_path"], None, 1000, strict=strict)
        top = FD.load_top_domains(gen["top1m"])
        t2 = time.perf_counter()
        feat = FD.featurize(tab, device, top, threads=threads)
        wsp = FD.DnsWordSpace(feat.cuts, feat.qpairs)
        dwc = count_pairs(feat.ip, feat.word_key, feat.weight)
        built = lda_pre(dwc)
        if device.type == "cuda":
            torch.cuda.synchronize()
        t3 = time.perf_counter()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    info = dict(events=events, synth_s=round(t1 - t0, 3), ingest_s=round(t2 - t1, 3),
                featurize_corpus_s=round(t3 - t2, 3))
    if return_names:
        return built.corpus, info, wsp.decode(built.word_keys)
    return built.corpus, info
