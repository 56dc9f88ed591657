"""Stages shared by the flow and DNS pipelines: corpus files, LDA, model export, model reload."""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch

from ..corpus.builder import BuiltCorpus, lda_pre
from ..corpus.csr import Corpus
from ..export import lda_post
from ..io import ldac
from ..models.lda.estimate import estimate


@dataclass
class ModelTables:
    """What the scorers consume: θ / φ and their row names (as written to the result files)."""
    doc_names: List[str]
    theta: np.ndarray          # [D, K]
    word_names: List[str]      # keys as written (strict: truncated to 20 bytes)
    phi: np.ndarray            # [V, K]
    # set when the tables were built in this process from its own vocabulary (compat=fixed): the word
    # key of every φ row and the key space that encodes them -- the flow scorer then maps event keys
    # to rows without decoding or hashing millions of word names
    word_keys: Optional[np.ndarray] = None
    key_space: Optional[object] = None

    def doc_index(self) -> dict:
        return {n: i for i, n in enumerate(self.doc_names)}      # later duplicates win (collectAsMap)

    def word_index(self) -> dict:
        return {n: i for i, n in enumerate(self.word_names)}

    @property
    def K(self) -> int:
        return int(self.theta.shape[1])

    def word_rows(self, names: List[str]) -> np.ndarray:
        """φ row of every word name (-1: not in word_results)."""
        idx = self.word_index()
        return np.fromiter((idx.get(n, -1) for n in names), dtype=np.int64, count=len(names))

    def compact(self, doc_rows: np.ndarray, word_rows: np.ndarray):
        """(θ, φ, doc rows, word rows) the score kernel indexes: the whole tables, rows unchanged."""
        return self.theta, self.phi, np.asarray(doc_rows, np.int64), np.asarray(word_rows, np.int64)


@dataclass
class ShardedTables:
    """The scorers' model in the row-sharded pipeline, nothing replicated: θ rows stay with the rank of
    their documents (global rows [doc_starts[r], doc_starts[r + 1])), φ rows with the rank of their
    vocabulary slice; the word name -> φ row map is hash-partitioned (``shardio.DistDict``, later rows
    win as in ``collectAsMap``).  A rank fetches only the θ / φ rows its own events reference
    (``shardio.fetch_rows``) -- the reference broadcasts the whole model to every executor
    (flow_post_lda.scala:112-123).  ``word_rows`` and ``compact`` are collective."""
    ctx: object
    theta: np.ndarray          # this rank's θ rows
    doc_starts: List[int]
    phi: np.ndarray            # this rank's φ rows (vocabulary slice)
    word_starts: List[int]
    words: object              # shardio.DistDict: word name as written -> global φ row

    @property
    def K(self) -> int:
        return int(self.theta.shape[1])

    def word_rows(self, names: List[str]) -> np.ndarray:
        return self.words.lookup(names)

    def compact(self, doc_rows: np.ndarray, word_rows: np.ndarray):
        """(θ rows, φ rows, local doc rows, local word rows): the distinct rows the given global rows
        reference, fetched from their owners, and the given rows renumbered into them (-1 kept)."""
        from ..parallel import shardio as SIO
        out = []
        for rows, tab, starts in ((doc_rows, self.theta, self.doc_starts), (word_rows, self.phi, self.word_starts)):
            rows = np.asarray(rows, np.int64)
            ok = rows >= 0
            u, inv = np.unique(rows[ok], return_inverse=True)
            got = SIO.fetch_rows(self.ctx, tab, starts, u)
            loc = np.full(rows.size, -1, np.int64)
            loc[ok] = inv
            out.append((got, loc))
        (th, dl), (ph, wl) = out
        return th, ph, dl, wl


def write_corpus_files(lpath: str, built: BuiltCorpus, doc_names: List[str], word_names: List[str]):
    ldac.write_words_dat(os.path.join(lpath, "words.dat"), word_names)
    ldac.write_doc_dat(os.path.join(lpath, "doc.dat"), doc_names)
    ldac.write_model_dat(os.path.join(lpath, "model.dat"), built.corpus)


def load_corpus_files(lpath: str):
    c = ldac.read_model_dat(os.path.join(lpath, "model.dat"))
    docs = ldac.read_index_file(os.path.join(lpath, "doc.dat"))
    words = ldac.read_index_file(os.path.join(lpath, "words.dat"))
    c.num_terms = max(c.num_terms, len(words))
    return c, docs, words


RANK_FILES_MAX_VALUES = 1 << 26
# lda_post writes its result files on a thread while the scoring stage runs from this many doc + word values
DEFER_POST_VALUES = 1 << 26


def run_lda(cfg, corpus: Corpus, dist=None, device=None, log=print, local_shard: bool = False, doc_offset: int = 0):
    outdir = cfg.lpath
    settings_path = os.path.join(outdir, "settings.txt")
    if dist is None or dist.rank == 0:
        ldac.write_settings(settings_path, cfg.settings)
    rank_files = cfg.rank_gamma
    if rank_files is None:
        # oni-lda-c's per-worker <rank>.beta / <rank>.gamma temporaries (README.md:121): on for multi-rank
        # runs while a worker's K x V beta text stays small (<= RANK_FILES_MAX_VALUES values; BASELINE
        # config 5's would be ~7 GB per rank); --rank-gamma forces them
        rank_files = dist is not None and dist.active and cfg.topics * corpus.num_terms <= RANK_FILES_MAX_VALUES
    return estimate(corpus, cfg.topics, cfg.alpha, cfg.settings, cfg.start, outdir, backend=cfg.backend,
                    device=device, dist=dist, seed=cfg.seed, resume=cfg.resume,
                    write_word_assignments=cfg.word_assignments,
                    write_rank_gamma=rank_files,
                    verbose=cfg.verbose, fault_at_iteration=cfg.extra.get("fault_at_iteration"),
                    defer_files=True, local_shard=local_shard, doc_offset=doc_offset)


def run_export(cfg, doc_names, gamma, word_names, log_beta, read_back: bool = False) -> ModelTables:
    """``read_back``: the tables as the scorers parse the files (what ``strict_tables`` computes, but
    from the writer's own formatting pass instead of a second one)."""
    th, ph, wn = lda_post.export(doc_names, gamma, word_names, log_beta,
                                 os.path.join(cfg.lpath, "doc_results.csv"),
                                 os.path.join(cfg.lpath, "word_results.csv"), strict=cfg.strict, read_back=read_back)
    return ModelTables(list(doc_names), th, wn, ph)


def load_model_tables(lpath: str) -> ModelTables:
    """Read doc_results.csv / word_results.csv exactly as the Scala scorers do."""
    dn, th = lda_post.read_results(os.path.join(lpath, "doc_results.csv"))
    wn, ph = lda_post.read_results(os.path.join(lpath, "word_results.csv"))
    return ModelTables(dn, th, wn, ph)


def strict_tables(mt: ModelTables, strict: bool = True) -> ModelTables:
    """θ/φ as the scorers see them after the text hand-off (Python-2 str -> toDouble).

    Applied in both compat modes: the result files are the stage contract, so an
    in-memory run and a run resumed from the files score identically."""
    from ..ops import native
    n = native.lib()
    return ModelTables(mt.doc_names, n.roundtrip_py2(np.ascontiguousarray(mt.theta)), mt.word_names,
                       n.roundtrip_py2(np.ascontiguousarray(mt.phi)))


def background(fn, name: str = "oni-writer"):
    """Run ``fn`` on a thread (the native writers release the GIL); returns the join callable a stage
    puts in ``result["_defer"]``, which re-raises the thread's exception."""
    import threading
    box = {}

    def body():
        from ..ops import native
        from ..utils.sched import background_priority
        background_priority()
        native.background_thread_budget()   # leaves the GPU-driving thread CPUs within the quota
        try:
            fn()
        except BaseException as e:  # noqa: BLE001 -- handed to the joiner
            box["err"] = e

    t = threading.Thread(target=body, name=name, daemon=True)
    t.start()

    def join():
        t.join()
        if "err" in box:
            raise box["err"]
    return join


def vocab_lookup(word_keys, word_names):
    """keys -> (names, index) through the built vocabulary (every doc_wc key is in it): a vectorized
    search instead of decoding the unique keys again -- a writer thread then holds the GIL only
    briefly while the lda stage drives the GPU."""
    wk = np.asarray(word_keys)
    srt = np.argsort(wk, kind="stable")
    sk = wk[srt]

    def lookup(keys):
        return word_names, srt[np.searchsorted(sk, np.asarray(keys))]
    return lookup


def doc_rows_of(doc_keys, n_keys: int) -> np.ndarray:
    """Doc row of every dictionary id (-1: not a document): the in-memory equivalent of looking the
    names up in doc_results.csv, when the documents are ``doc_keys`` in row order."""
    rows = np.full(int(n_keys), -1, np.int64)
    dk = np.asarray(doc_keys, np.int64)
    rows[dk] = np.arange(dk.size, dtype=np.int64)
    return rows


def save_json(path: str, obj):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))


def load_json(path: str):
    with open(path) as f:
        return json.load(f)
