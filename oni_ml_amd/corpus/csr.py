"""Document-word corpus in CSR form (the in-memory equivalent of lda-c's model.dat).

Reference contract: lda_pre.py:84-94 writes one line per document,
``N w:c w:c ...``; oni-lda-c's read_data parses it into {words, counts, length,
total} with num_terms = max(word id)+1.  Here the corpus is a
pair of flat arrays plus row offsets, and a word-major (CSC) permutation used by
the deterministic sufficient-statistics kernel.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch


@dataclass
class Corpus:
    doc_ptr: np.ndarray          # int64 [D+1]
    word_idx: np.ndarray         # int32 [nnz]
    counts: np.ndarray           # int64 [nnz]
    num_terms: int
    doc_names: Optional[List[str]] = None
    word_names: Optional[List[str]] = None
    meta: dict = field(default_factory=dict)

    def __post_init__(self):
        self.doc_ptr = np.ascontiguousarray(self.doc_ptr, dtype=np.int64)
        self.word_idx = np.ascontiguousarray(self.word_idx, dtype=np.int32)
        self.counts = np.ascontiguousarray(self.counts, dtype=np.int64)
        if self.doc_ptr.ndim != 1 or self.doc_ptr[0] != 0 or self.doc_ptr[-1] != self.word_idx.size:
            raise ValueError("inconsistent CSR doc_ptr")
        if self.word_idx.size != self.counts.size:
            raise ValueError("word_idx / counts length mismatch")
        if self.word_idx.size and (self.word_idx.min() < 0 or self.word_idx.max() >= self.num_terms):
            raise ValueError("word index out of range")

    @property
    def num_docs(self) -> int:
        return int(self.doc_ptr.size - 1)

    @property
    def nnz(self) -> int:
        return int(self.word_idx.size)

    def lengths(self) -> np.ndarray:
        return np.diff(self.doc_ptr)

    def totals(self) -> np.ndarray:
        return np.add.reduceat(self.counts, self.doc_ptr[:-1]) if self.nnz else np.zeros(self.num_docs, np.int64)

    def slice_docs(self, d0: int, d1: int) -> "Corpus":
        """Contiguous shard [d0, d1) with local doc ids (same vocabulary)."""
        a, b = int(self.doc_ptr[d0]), int(self.doc_ptr[d1])
        return Corpus(
            doc_ptr=self.doc_ptr[d0:d1 + 1] - a,
            word_idx=self.word_idx[a:b],
            counts=self.counts[a:b],
            num_terms=self.num_terms,
            doc_names=self.doc_names[d0:d1] if self.doc_names is not None else None,
            word_names=self.word_names,
            meta=dict(self.meta, shard=(d0, d1)),
        )

    @staticmethod
    def from_docs(docs, num_terms=None) -> "Corpus":
        """docs: list of [(word, count), ...] (tests / small inputs)."""
        ptr = [0]
        w, c = [], []
        for d in docs:
            for wi, ci in d:
                w.append(wi)
                c.append(ci)
            ptr.append(len(w))
        w = np.asarray(w, np.int32)
        nt = int(num_terms if num_terms is not None else (w.max() + 1 if w.size else 0))
        return Corpus(np.asarray(ptr, np.int64), w, np.asarray(c, np.int64), nt)


@dataclass
class DeviceCorpus:
    """Corpus resident on one device: CSR + CSC (word-major) + length buckets."""
    doc_ptr: torch.Tensor        # int32 [D+1]
    word_idx: torch.Tensor       # int32 [nnz]
    counts: torch.Tensor         # float32 [nnz]
    word_ptr: torch.Tensor       # int32 [V+1]
    csc_ent: torch.Tensor        # int32 [nnz]  CSR entry of each CSC slot
    csc_doc: torch.Tensor        # int32 [nnz]
    num_docs: int
    num_terms: int
    nnz: int
    doc_len: np.ndarray          # host copy of lengths
    word_len: np.ndarray         # host copy of entries per word

    @staticmethod
    def build(c: Corpus, device) -> "DeviceCorpus":
        if c.nnz >= 2**31 - 1:
            raise ValueError("nnz exceeds int32 offsets; shard the corpus")
        if torch.device(device).type == "cuda":
            return DeviceCorpus._build_device(c, torch.device(device))
        D, V = c.num_docs, c.num_terms
        lens = c.lengths()
        doc_of = np.repeat(np.arange(D, dtype=np.int32), lens)
        # stable word-major permutation: entries of a word in doc order
        perm = np.argsort(c.word_idx, kind="stable").astype(np.int32)
        wlen = np.bincount(c.word_idx, minlength=V).astype(np.int64)
        wptr = np.zeros(V + 1, np.int64)
        np.cumsum(wlen, out=wptr[1:])
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)
        return DeviceCorpus(
            doc_ptr=t(c.doc_ptr, torch.int32),
            word_idx=t(c.word_idx, torch.int32),
            counts=t(c.counts.astype(np.float32), torch.float32),
            word_ptr=t(wptr, torch.int32),
            csc_ent=t(perm, torch.int32),
            csc_doc=t(doc_of[perm], torch.int32),
            num_docs=D, num_terms=V, nnz=c.nnz,
            doc_len=lens.astype(np.int64), word_len=wlen,
        )

    @staticmethod
    def _build_device(c: Corpus, dev) -> "DeviceCorpus":
        """The CSC permutation on the GPU: one stable radix sort of the word ids (nnz entries), the
        column pointer from a searchsorted -- instead of a host argsort of nnz entries (the engine's
        setup cost, seconds at the 30-day scale)."""
        D, V = c.num_docs, c.num_terms
        lens = c.lengths()
        ptr = torch.from_numpy(c.doc_ptr).to(dev)
        w = torch.from_numpy(c.word_idx).to(dev)
        cnt = torch.from_numpy(c.counts).to(dev).to(torch.float32)
        ws, perm = torch.sort(w, stable=True)
        wptr = torch.searchsorted(ws, torch.arange(V + 1, device=dev, dtype=ws.dtype))
        from ..ops import sortgroup as SG
        doc_of = SG.segment_ids(ptr[1:] - ptr[:-1], total=c.nnz).to(torch.int32)   # (no repeat_interleave)
        wlen = (wptr[1:] - wptr[:-1]).cpu().numpy().astype(np.int64)
        return DeviceCorpus(
            doc_ptr=ptr.to(torch.int32), word_idx=w.to(torch.int32), counts=cnt,
            word_ptr=wptr.to(torch.int32), csc_ent=perm.to(torch.int32), csc_doc=SG.gather(doc_of, perm),
            num_docs=D, num_terms=V, nnz=c.nnz, doc_len=lens.astype(np.int64), word_len=wlen,
        )
