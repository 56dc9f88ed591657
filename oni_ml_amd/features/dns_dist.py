"""Row-sharded DNS featurization over N ranks (dns_pre_lda.scala:141-334 on Spark executors,
ml_ops.sh:57).

* ingest -- rank r reads rows [R r / N, R (r + 1) / N) of the selected parquet inputs taken as one
  table (only the row groups holding them), then applies the reference's row rules to its slice;
  the analyst-feedback rows (last in the single-process order) go to the last rank;
* the five cut sets -- every rank's weighted histogram of each feature (values > 0 only for the
  three quintile features) all-gathered and merged, the cut rule on the merged histogram;
* dictionaries -- ip_dst and the "qry_type_qry_rcode" pairs in global first-appearance order
  (``shardio.first_appearance``);
* (ip_dst, word) counts -- local, routed by corpus/sharded.py.

Identical to one process featurizing the whole day (tests/test_sharded_pipeline.py).
"""
from __future__ import annotations

import numpy as np
import torch

from ..corpus.builder import count_pairs
from ..ops import native
from ..parallel import shardio as SIO
from . import dns as FD
from .dns_data import COUNTRY_CODES, SPECIAL_DOMAIN
from .flow_dist import merged_hist
from .quantiles import DECILES, QUINTILES, ecdf_cuts_from_hist


def load_dns_sharded(ctx, dns_path: str, feedback_path=None, dupfactor: int = 1000, strict: bool = True) -> FD.DnsTable:
    N, r = SIO.world(ctx), SIO.rank(ctx)
    total = FD.dns_total_rows(dns_path, strict)
    lo, hi = total * r // N, total * (r + 1) // N
    tables = FD.load_dns_rows(dns_path, lo, hi, strict)
    fb = FD.read_dns_feedback(feedback_path) if (feedback_path and r == N - 1) else []
    return FD.table_from_arrow(tables, fb, dupfactor)


def _arrow_bytes(arr):
    data, off = FD._offsets(arr)
    return np.frombuffer(memoryview(data), np.uint8) if len(data) else np.zeros(0, np.uint8), off


def global_dictionary(ctx, arr):
    """(global names, global id of every row) for an Arrow string column."""
    _, pc, _ = FD._pa()
    d = pc.dictionary_encode(arr)
    ids = d.indices.to_numpy(zero_copy_only=False).astype(np.int64)
    data, off = _arrow_bytes(d.dictionary)
    names, lmap = SIO.first_appearance(ctx, data, off)
    return names, lmap[ids] if ids.size else ids, lmap


def _values(tab: FD.DnsTable, n: int, top_domains, device, threads: int):
    data, off = FD._offsets(tab.column("dns_qry_name", n))
    F = native.lib().dns_features(data, off, list(COUNTRY_CODES), list(top_domains), SPECIAL_DOMAIN, threads)
    vals = dict(
        frame_len=torch.from_numpy(tab.frame_len[:n]).to(device),
        unix_tstamp=torch.from_numpy(tab.unix_tstamp[:n]).to(device),
        subdomain_length=torch.from_numpy(F["subdomain_length"].astype(np.float64)).to(device),
        entropy=torch.from_numpy(F["entropy"]).to(device),
        num_periods=torch.from_numpy(F["num_periods"].astype(np.float64)).to(device),
    )
    return F, vals, torch.from_numpy(tab.weight[:n]).to(device)


def _cuts(ctx, vals, w) -> dict:
    cuts_t = {}
    for k, q in (("unix_tstamp", DECILES), ("frame_len", DECILES)):
        cuts_t[k] = ecdf_cuts_from_hist(*merged_hist(ctx, vals[k], w), q)
    for k in ("subdomain_length", "entropy", "num_periods"):
        m = vals[k] > 0
        cuts_t[k] = ecdf_cuts_from_hist(*merged_hist(ctx, vals[k][m], w[m]), QUINTILES)
    return cuts_t


def global_cuts(ctx, tab: FD.DnsTable, top_domains, device, raw_only: bool = False, threads: int = 8) -> dict:
    """The five cut sets over every rank's rows (raw_only: without the feedback rows, dns_post_lda.scala)."""
    _, vals, w = _values(tab, tab.n_raw if raw_only else tab.n, top_domains, torch.device(device), threads)
    return {k: v.cpu().numpy() for k, v in _cuts(ctx, vals, w).items()}


def featurize_sharded(ctx, tab: FD.DnsTable, device, top_domains, cuts=None, threads: int = 8):
    """This rank's rows -> (sections [(ip, word) counts, global ids], ip names, local ip id -> global id,
    word space, cuts).  ``cuts``: fixed cuts instead of the global ECDF ones."""
    device = torch.device(device)
    n = tab.n
    F, vals, w = _values(tab, n, top_domains, device, threads)
    if cuts is None:
        cuts_t = _cuts(ctx, vals, w)
    else:
        cuts_t = {k: torch.as_tensor(np.asarray(v, np.float64), device=device) for k, v in cuts.items()}
    bins = {k: (vals[k].unsqueeze(-1) > cuts_t[k].unsqueeze(0)).sum(-1) for k in vals}
    _, pc, _ = FD._pa()
    qnames, qid, _ = global_dictionary(
        ctx, pc.binary_join_element_wise(tab.column("dns_qry_type", n), tab.column("dns_qry_rcode", n), "_"))
    qnames = qnames.all()
    top = torch.from_numpy(F["top_domain"].astype(np.int64)).to(device)
    key = top
    radix = {k: len(cuts_t[k]) + 1 for k in FD.DnsWordSpace.ORDER}
    for k in FD.DnsWordSpace.ORDER:
        key = key * radix[k] + bins[k]
    key = key * max(1, len(qnames)) + torch.from_numpy(qid).to(device)
    ip_names, ip_gid, ip_map = global_dictionary(ctx, tab.column("ip_dst", n))
    ip = torch.from_numpy(ip_gid).to(device)
    cuts_np = {k: v.cpu().numpy() for k, v in cuts_t.items()}
    wsp = FD.DnsWordSpace(cuts_np, qnames)
    return [count_pairs(ip, key, w)], ip_names, ip_map, wsp, cuts_np
