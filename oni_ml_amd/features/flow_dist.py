"""Row-sharded netflow featurization over N ranks (the reference's Spark executors, SURVEY.md P1 /
§5.8 "Featurization"; flow_pre_lda.scala:280-290 quantile jobs, :366-380 reduceByKey counts).

Every rank ingests only its byte range of the input (a line belongs to the range holding its first
byte, so the N ranges partition the rows exactly and in file order), and the ranks meet only where
the single-process pipeline looks at all rows at once -- always through tensor collectives
(parallel/shardio.py), never pickled objects:

* IP dictionary -- ids in global first-appearance order: every rank's dictionary (local
  first-appearance order) packed into fixed-width integer rows, hash-partitioned over the ranks and
  merged by each owner with ``shardio.unique_rows`` (``shardio.first_appearance``);
* ECDF cuts -- each rank's weighted value histogram (distinct values, summed integer weights) is
  all-gathered and merged; the cut rule runs on the merged histogram, which is exactly the weighted
  multiset the single-process ecdf_cuts sees;
* word space -- the union of the ranks' distinct word_port values;
* (ip, word) counts -- each rank counts its own rows (reduceByKey); the partial counts are NOT
  replicated: corpus/sharded.py routes them to the rank owning each document's id range.

The result (cuts, word space, doc_wc and hence doc.dat / words.dat / model.dat) is identical to
one process featurizing all rows (tests/test_flow_dist.py).  Analyst-feedback rows come last in the
single-process row order, so the last rank ingests them.
"""
from __future__ import annotations

import os
from typing import List, Tuple

import numpy as np
import torch

from ..corpus.builder import DocWordCounts, count_pairs, segment_sums
from ..ops import native
from ..parallel import shardio as SIO
from . import flow as FF
from .quantiles import DECILES, QUINTILES, ecdf_cuts_from_hist


def byte_ranges(paths: List[str], world: int, rank: int) -> List[Tuple[str, int, int]]:
    """This rank's pieces (path, begin, end) of the files' concatenated byte space, split evenly."""
    sizes = [os.path.getsize(p) for p in paths]
    total = sum(sizes)
    lo, hi = total * rank // world, total * (rank + 1) // world
    out, off = [], 0
    for p, s in zip(paths, sizes):
        b, e = max(lo, off), min(hi, off + s)
        if b < e:
            out.append((p, b - off, e - off))
        off += s
    return out


def _first_line(path: str) -> str:
    with open(path, "rb") as f:
        line = f.readline().decode("utf-8", errors="surrogateescape")
    return line.rstrip("\n").rstrip("\r")


def load_flow_sharded(ctx, flow_path: str, feedback_path=None, dupfactor: int = 1000, threads: int = 8) -> FF.FlowTable:
    """This rank's rows of FLOW_PATH (+ the feedback rows on the last rank)."""
    paths = FF.list_inputs(flow_path)
    if not paths:
        raise FileNotFoundError(f"no flow input under {flow_path!r}")
    header = _first_line(paths[0])
    t = native.lib().TextTable(FF.NCOLS, FF.NUMERIC, [[FF.C_SIP, FF.C_DIP]])
    for p, b, e in byte_ranges(paths, ctx.world_size, ctx.rank):
        t.load_range(p, b, e, header, True, threads)
    n_raw = t.num_rows
    if ctx.rank == ctx.world_size - 1 and feedback_path:
        fb = FF.read_flow_feedback(feedback_path)
        if fb:
            t.append_text("\n".join(fb), weight=int(dupfactor), threads=threads)
    return FF.FlowTable(t, n_raw, t.num_rows - n_raw, int(dupfactor))


def global_ip_dictionary(ctx, ft: FF.FlowTable):
    """(global names table in first-appearance order, local id -> global id)."""
    data, off = ft.table.dict_bytes(0)
    return SIO.first_appearance(ctx, data, off)


def merged_hist(ctx, values: torch.Tensor, w: torch.Tensor):
    """Global weighted histogram (sorted distinct values, summed weights) of every rank's values."""
    u, c = segment_sums(values.to(torch.float64).reshape(-1), w.to(torch.int64).reshape(-1))
    us = SIO.allgather_array(ctx, u.cpu().numpy())
    cs = SIO.allgather_array(ctx, c.cpu().numpy())
    dev = values.device
    return segment_sums(torch.from_numpy(np.concatenate(us)).to(dev), torch.from_numpy(np.concatenate(cs)).to(dev))


def global_cuts(ctx, cols: dict, w: torch.Tensor, device) -> dict:
    time = (cols["hour"] + cols["minute"] / 60) + cols["second"] / 3600
    qs = dict(time=DECILES, ibyt=DECILES, ipkt=QUINTILES)
    out = {}
    for name, v in (("time", time), ("ibyt", cols["ibyt"]), ("ipkt", cols["ipkt"])):
        mu, mc = merged_hist(ctx, v, w)
        out[name] = ecdf_cuts_from_hist(mu, mc, qs[name])
    return out


def table_columns(ft: FF.FlowTable, n: int, device) -> Tuple[dict, torch.Tensor]:
    t = ft.table

    def col(c):
        return torch.from_numpy(t.numeric(c)[:n]).to(device)
    cols = dict(hour=col(FF.C_HOUR), minute=col(FF.C_MIN), second=col(FF.C_SEC), a=col(FF.C_A), b=col(FF.C_B),
                ipkt=col(FF.C_IPKT), ibyt=col(FF.C_IBYT))
    return cols, torch.from_numpy(t.weights()[:n].astype(np.int64)).to(device)


def featurize_sharded(ctx, ft: FF.FlowTable, device, cuts=None):
    """Distributed pre-LDA featurization of this rank's rows.

    Returns (sections, names, ip_map, ws, cuts): the source- and destination-side (ip, word) counts
    of this rank's rows (global ip ids, sorted by (ip, word)); the global IP dictionary; this rank's
    local -> global ip ids; the word space and the cuts (identical on every rank and to the
    single-process pipeline).  ``cuts``: fixed cuts (the CUT setting) instead of the global ECDF."""
    device = torch.device(device)
    t = ft.table
    n = ft.n
    cols, w = table_columns(ft, n, device)
    if cuts is None:
        cuts = global_cuts(ctx, cols, w, device)
    else:
        cuts = {k: torch.as_tensor(np.asarray(v, np.float64), device=device) for k, v in cuts.items()}
    out = FF._flow_words(cols, cuts, device)
    ports = np.unique(np.concatenate(SIO.allgather_array(ctx, torch.unique(out["word_port"]).cpu().numpy())))
    ws = FF.FlowWordSpace(ports, len(cuts["time"]) + 1, len(cuts["ibyt"]) + 1, len(cuts["ipkt"]) + 1)
    names, gmap = global_ip_dictionary(ctx, ft)
    gm = torch.from_numpy(gmap).to(device)
    sip = gm[torch.from_numpy(t.dict_ids(FF.C_SIP)[:n].astype(np.int64)).to(device)]
    dip = gm[torch.from_numpy(t.dict_ids(FF.C_DIP)[:n].astype(np.int64)).to(device)]
    feat = FF.FlowFeatures(time=out["time"], time_bin=out["time_bin"], ibyt_bin=out["ibyt_bin"],
                           ipkt_bin=out["ipkt_bin"], word_port=out["word_port"], src_prefix=out["src_prefix"],
                           dst_prefix=out["dst_prefix"], sip=sip, dip=dip, weight=w,
                           cuts={k: v.cpu().numpy() for k, v in cuts.items()}, rows=np.arange(n, dtype=np.int64))
    src, dst = FF.word_keys(feat, ws)
    sections = [count_pairs(sip, src, w), count_pairs(dip, dst, w)]
    return sections, names, gmap, ws, feat.cuts
