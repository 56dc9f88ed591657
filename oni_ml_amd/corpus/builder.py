"""Corpus builder: (doc, word) event pairs -> doc_wc -> lda-c corpus (lda_pre.py equivalent).

Reference pipeline:
* the pre-LDA stage counts (ip, word) pairs with reduceByKey -- twice for flow
  (source side and destination side, flow_pre_lda.scala:366-373) and unions the
  two results WITHOUT merging, so one (ip, word) can appear twice;
* lda_pre.py reads the resulting ``ip,word,count`` lines and assigns word ids
  in first-appearance order (0-based, words.dat), doc ids in first-appearance
  order (1-based, doc.dat), and writes each doc's entries in line order
  (model.dat).

Here the counting is a sort-based group-by on packed int64 keys on the device
(torch.unique), and the lda_pre dictionaries are first-appearance ranks
computed with scatter-min; nothing is materialised as text unless asked.
The reference's doc_wc line order is Spark hash-partition order (not
reproducible); ours is deterministic: section by section, pairs sorted by
(ip dictionary id, word key).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import sortgroup as SG
from .csr import Corpus

_SHIFT = 32


@dataclass
class DocWordCounts:
    """doc_wc in line order (device tensors)."""
    doc: torch.Tensor      # int64 ip/doc dictionary ids
    word: torch.Tensor     # int64 word keys
    count: torch.Tensor    # int64

    @property
    def n(self) -> int:
        return int(self.doc.numel())

    def to_host(self) -> "DocWordCounts":
        """The same counts as host tensors.  The lda_pre text writer runs on a thread beside the EM; a
        device-to-host copy issued from that thread waited for the EM batch in flight and held up the
        enqueue of the next one (the lda stage 69 -> 114 ms, profiles/r6m_lda_stage_ab.json), so the
        pipeline copies on its own thread before it starts the writer."""
        return DocWordCounts(self.doc.cpu(), self.word.cpu(), self.count.cpu())


def count_pairs(doc: torch.Tensor, word: torch.Tensor, weight: Optional[torch.Tensor] = None) -> DocWordCounts:
    """reduceByKey((doc, word), +weight) with output sorted by (doc, word)."""
    if doc.numel() and (int(word.min()) < 0 or int(word.max()) >= (1 << _SHIFT)):
        raise ValueError("word keys must fit in 32 bits")
    pk = (doc.to(torch.int64) << _SHIFT) | word.to(torch.int64)
    if weight is None:
        uniq, cnt = SG.unique(pk, return_counts=True)
    else:
        uniq, cnt = segment_sums(pk, weight.to(device=pk.device, dtype=torch.int64))
    return DocWordCounts(uniq >> _SHIFT, uniq & ((1 << _SHIFT) - 1), cnt)


def segment_sums(keys: torch.Tensor, w: torch.Tensor):
    """(sorted distinct keys, sum of w per key) by a radix sort and a prefix sum -- no atomics, so
    heavily repeated keys (a handful of port words, hour-of-day values) cost nothing extra; an
    int64 index_add_ over them serialises on a few contended addresses (ops/sortgroup.py)."""
    return SG.segment_sums(keys, w)


def concat(parts: Sequence[DocWordCounts], merge: bool = False) -> DocWordCounts:
    """Union of sections; merge=True sums duplicate (doc, word) pairs across sections."""
    doc = torch.cat([p.doc for p in parts])
    word = torch.cat([p.word for p in parts])
    cnt = torch.cat([p.count for p in parts])
    if merge:
        return count_pairs(doc, word, cnt)
    return DocWordCounts(doc, word, cnt)


def _first_appearance_ids(keys: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """ids[i] = rank of keys[i]'s first appearance; returns (ids, distinct keys in rank order)."""
    # stable sort: the first element of each run of equal keys is the key's first appearance
    # (ops/sortgroup.py: the group of every sorted position from a prefix sum, no repeat_interleave)
    sk, perm = SG.sort_stable(keys)
    grp, G = SG.run_ids(sk)
    st = SG.run_starts(grp, G)[:-1]
    first = SG.gather(perm, st)
    inv = torch.empty_like(perm)
    inv[perm] = grp
    order = torch.sort(first).indices          # first appearances are distinct: any sort is the stable one
    rank = torch.empty_like(order)
    rank[order] = torch.arange(order.numel(), device=keys.device)
    return SG.gather(rank, inv), SG.gather(SG.gather(sk, st), order)


@dataclass
class BuiltCorpus:
    corpus: Corpus
    doc_keys: np.ndarray     # [D] ip dictionary id of each doc (doc.dat order)
    word_keys: np.ndarray    # [V] word key of each word id (words.dat order)


def lda_pre(dwc: DocWordCounts) -> BuiltCorpus:
    """lda_pre.py semantics on device: first-appearance word / doc ids, entries grouped by doc in line order."""
    if dwc.n == 0:
        raise ValueError("empty doc_wc: no (ip, word) pairs survived featurization")
    wid, wkeys = _first_appearance_ids(dwc.word)
    did, dkeys = _first_appearance_ids(dwc.doc)
    order = torch.sort(did, stable=True).indices
    d_sorted = SG.gather(did, order)
    D = int(dkeys.numel())
    # d_sorted is sorted: the CSR offsets are a binary search per document (a bincount would be
    # an atomic histogram over the entries)
    ptr = torch.searchsorted(d_sorted, torch.arange(D + 1, device=d_sorted.device, dtype=d_sorted.dtype))
    corpus = Corpus(
        doc_ptr=ptr.cpu().numpy(),
        word_idx=SG.gather(wid, order).to(torch.int32).cpu().numpy(),
        counts=SG.gather(dwc.count, order).cpu().numpy(),
        num_terms=int(wkeys.numel()),
    )
    return BuiltCorpus(corpus, dkeys.cpu().numpy(), wkeys.cpu().numpy())


def lda_pre_reference(lines: List[Tuple[str, str, int]]):
    """Literal lda_pre.py (test oracle): returns (words list, docs list, model lines)."""
    wcdict, words = {}, []
    for ip, w, c in lines:
        if w not in wcdict:
            wcdict[w] = len(words)
            words.append(w)
    docdict, docs = {}, []
    for ip, w, c in lines:
        if ip in docdict:
            docdict[ip][1] += 1
            docdict[ip][2].append(" %s:%s" % (wcdict[w], c))
        else:
            docdict[ip] = [len(docs) + 1, 1, [" %s:%s" % (wcdict[w], c)]]
            docs.append(ip)
    model = ["%s%s" % (docdict[ip][1], "".join(docdict[ip][2])) for ip in docs]
    return words, docs, model


def read_doc_wc(path: str, threads: int = 8):
    """Parse a doc_wc.dat (``ip,word,count``) with the C++ ingest: returns (DocWordCounts on CPU, ip names, word names)."""
    from ..ops import native
    t = native.lib().TextTable(3, [2], [[0], [1]])
    t.load_files([path], drop_header=False, threads=threads)
    dwc = DocWordCounts(torch.from_numpy(t.dict_ids(0).astype(np.int64)),
                        torch.from_numpy(t.dict_ids(1).astype(np.int64)),
                        torch.from_numpy(t.numeric(2).astype(np.int64)))
    return dwc, t.dict_names(0), t.dict_names(1)


def write_doc_wc(path: str, dwc: DocWordCounts, doc_names: Sequence[str], word_names_of_key):
    """Write doc_wc.dat lines ``ip,word,count`` (word_names_of_key: callable keys -> (names list, index array))."""
    from ..ops import native
    names, idx = word_names_of_key(dwc.word.cpu().numpy())
    native.lib().write_rows(path, None, [("dict", list(doc_names), dwc.doc.cpu().numpy().astype(np.int32)),
                                         ("dict", names, idx.astype(np.int32)),
                                         ("int", dwc.count.cpu().numpy())], n=dwc.n)
