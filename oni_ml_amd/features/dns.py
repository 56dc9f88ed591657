"""DNS featurization: parquet -> per-query words -> (ip_dst, word) counts.

Reference: dns_pre_lda.scala (pre-LDA) and dns_post_lda.scala:108-297 (repeated
before scoring); SURVEY.md C6a-C6i, C7b.

* input: Hive/parquet paths (comma-separated DNS_PATH); the reference reads
  path 0 and then only paths with index > 1, silently skipping index 1
  (dns_pre_lda.scala:142-148) -- reproduced in compat=strict;
* rows with null frame_len / unix_tstamp are dropped; each row is printed with
  Row.mkString(",") (nulls become "null") and kept only if it splits back
  into exactly 8 fields (a comma inside any value drops the row);
* analyst feedback: dns_scores.csv rows with dns_sev == 3 (24-col schema,
  dns_pre_lda.scala:84-139), weight DUPFACTOR;
* per-name features (domain / subdomain / lengths / Scala-order entropy /
  top-1m flag) in the multithreaded C++ parser (csrc/native/dns.cpp);
* cuts: deciles of unix_tstamp and frame_len, quintiles of subdomain length,
  entropy and label count over values > 0 only; bins on the device;
* word = top _ bin(frame_len) _ bin(tstamp) _ bin(sublen) _ bin(entropy) _
  bin(labels) _ qry_type _ qry_rcode (integers, dns_pre_lda.scala:320-327).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..ops import native
from .dns_data import COUNTRY_CODES, SPECIAL_DOMAIN
from .quantiles import DECILES, QUINTILES, ecdf_cuts

from .dns_io import (  # noqa: F401  (re-exported: the torch-free ingest)
    COLUMNS, FEEDBACK_IDX, _pa, select_paths, _java_split_len, read_dns_feedback, _java_double, DnsTable,
    _arrow_strings, load_dns, _parquet_files, load_dns_rows, dns_total_rows, table_from_arrow, load_top_domains,
    _offsets, arrow_dictionary_encode, host_features)


@dataclass
class DnsFeatures:
    rows: np.ndarray                  # table rows featurized
    ip: torch.Tensor                  # int64 ip_dst dictionary id
    ip_names: List[str]
    word_key: torch.Tensor            # int64
    weight: torch.Tensor
    bins: Dict[str, torch.Tensor]
    cuts: Dict[str, np.ndarray]
    host: dict                        # C++ name features (host arrays)
    qpairs: List[str]                 # "type_rcode" dictionary


def dictionary_encode(values: List[str]):
    """First-appearance ids + names."""
    d = {}
    ids = np.empty(len(values), np.int32)
    for i, v in enumerate(values):
        j = d.get(v)
        if j is None:
            j = len(d)
            d[v] = j
        ids[i] = j
    return ids, list(d.keys())


def featurize(tab: DnsTable, device, top_domains: Sequence[str], cuts: Optional[Dict[str, np.ndarray]] = None,
              raw_only: bool = False, threads: int = 8, host: Optional[dict] = None) -> DnsFeatures:
    """``host``: the host features (``host_features``, or what ``featurize`` returned) of a prefix-compatible
    row set of the same table (the prefetch thread's or dns_pre's, over every row, reused by dns_post over
    the raw rows): the per-row arrays are cut to this call's rows; the dictionaries are first-appearance over
    the rows, so a prefix keeps its ids (and its names are a prefix of the names)."""
    device = torch.device(device)
    n = tab.n_raw if raw_only else tab.n
    if host is not None and len(host["entropy"]) >= n:
        m = len(host["entropy"])
        F = {k: (v[:n] if isinstance(v, np.ndarray) and v.ndim == 1 and len(v) == m else v) for k, v in host.items()}
        if n < m:   # a prefix: its dictionaries' names are the names up to its largest id
            for ids, names in (("_qid", "_qnames"), ("_ip_ids", "_ip_names")):
                F[names] = F[names][:int(F[ids].max()) + 1] if n else []
    else:
        F = host_features(tab, top_domains, threads, n)
    w = torch.from_numpy(tab.weight[:n]).to(device)
    vals = dict(
        frame_len=torch.from_numpy(tab.frame_len[:n]).to(device),
        unix_tstamp=torch.from_numpy(tab.unix_tstamp[:n]).to(device),
        subdomain_length=torch.from_numpy(F["subdomain_length"].astype(np.float64)).to(device),
        entropy=torch.from_numpy(F["entropy"]).to(device),
        num_periods=torch.from_numpy(F["num_periods"].astype(np.float64)).to(device),
    )
    if cuts is None and host is not None and n in host.get("_cuts", {}):
        # the prefetch child's host cuts for these rows (features/cuts_host.py: the same rule, same bits)
        cuts_t = {k: torch.as_tensor(np.asarray(v, np.float64), device=device) for k, v in host["_cuts"][n].items()}
    elif cuts is None:
        cuts_t = {}
        for k, q in (("unix_tstamp", DECILES), ("frame_len", DECILES)):
            cuts_t[k] = ecdf_cuts(vals[k], q, w)
        for k in ("subdomain_length", "entropy", "num_periods"):
            m = vals[k] > 0
            cuts_t[k] = ecdf_cuts(vals[k][m], QUINTILES, w[m])
    else:
        cuts_t = {k: torch.as_tensor(np.asarray(v, np.float64), device=device) for k, v in cuts.items()}
    bins = {k: (vals[k].unsqueeze(-1) > cuts_t[k].unsqueeze(0)).sum(-1) for k in vals}
    qid, qnames = F["_qid"], F["_qnames"]
    top = torch.from_numpy(F["top_domain"].astype(np.int64)).to(device)
    key = top
    radix = dict(frame_len=len(cuts_t["frame_len"]) + 1, unix_tstamp=len(cuts_t["unix_tstamp"]) + 1,
                 subdomain_length=len(cuts_t["subdomain_length"]) + 1, entropy=len(cuts_t["entropy"]) + 1,
                 num_periods=len(cuts_t["num_periods"]) + 1)
    for k in ("frame_len", "unix_tstamp", "subdomain_length", "entropy", "num_periods"):
        key = key * radix[k] + bins[k]
    key = key * max(1, len(qnames)) + torch.from_numpy(qid.astype(np.int64)).to(device)
    ip_ids, ip_names = F["_ip_ids"], F["_ip_names"]
    return DnsFeatures(rows=np.arange(n, dtype=np.int64), ip=torch.from_numpy(ip_ids.astype(np.int64)).to(device),
                       ip_names=ip_names, word_key=key, weight=w, bins=bins,
                       cuts={k: v.cpu().numpy() for k, v in cuts_t.items()}, host=F, qpairs=qnames)


class DnsWordSpace:
    """Decodes DNS word keys to the reference's word strings."""

    ORDER = ("frame_len", "unix_tstamp", "subdomain_length", "entropy", "num_periods")

    def __init__(self, cuts: Dict[str, np.ndarray], qpairs: List[str]):
        self.radix = [len(cuts[k]) + 1 for k in self.ORDER]
        self.qpairs = list(qpairs)

    def decode(self, keys: np.ndarray) -> List[str]:
        """Word strings of ``keys`` (csrc/native/bind_native.cpp radix_word_names; ``decode_py`` is the
        Python form, its test oracle)."""
        from ..ops import native
        return native.lib().radix_word_names(np.asarray(keys, np.int64), [int(r) for r in self.radix],
                                             list(self.qpairs))

    def decode_py(self, keys: np.ndarray) -> List[str]:
        k = np.asarray(keys, np.int64)
        nq = max(1, len(self.qpairs))
        q = k % nq
        k = k // nq
        parts = []
        for r in reversed(self.radix):
            parts.append(k % r)
            k = k // r
        top = k
        parts = parts[::-1]
        # column-wise str conversion, then one join per word (the per-element int() / indexing of a
        # row-wise loop cost ~1 us per word on the DNS day's 42 k words)
        cols = [list(map(str, top.tolist()))] + [list(map(str, p.tolist())) for p in parts]
        qp = self.qpairs
        cols.append([qp[i] for i in q.tolist()])
        return ["_".join(t) for t in zip(*cols)]
