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

    def doc_index(self) -> dict:
        return {n: i for i, n in enumerate(self.doc_names)}      # later duplicates win (collectAsMap)

    def word_index(self) -> dict:
        return {n: i for i, n in enumerate(self.word_names)}


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


def run_lda(cfg, corpus: Corpus, dist=None, device=None, log=print, local_shard: bool = False, doc_offset: int = 0):
    outdir = cfg.lpath
    settings_path = os.path.join(outdir, "settings.txt")
    if dist is None or dist.rank == 0:
        ldac.write_settings(settings_path, cfg.settings)
    return estimate(corpus, cfg.topics, cfg.alpha, cfg.settings, cfg.start, outdir, backend=cfg.backend,
                    device=device, dist=dist, seed=cfg.seed, resume=cfg.resume,
                    write_word_assignments=cfg.word_assignments,
                    write_rank_gamma=(cfg.rank_gamma if cfg.rank_gamma is not None
                                      else dist is not None and dist.active),
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


def map_names(names: List[str], index: dict, device) -> torch.Tensor:
    """Name list -> row ids through a {name: row} map (-1 when absent), as a device int64 tensor."""
    ids = np.fromiter((index.get(n, -1) for n in names), dtype=np.int64, count=len(names))
    return torch.from_numpy(ids).to(device)


def save_json(path: str, obj):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))


def load_json(path: str):
    with open(path) as f:
        return json.load(f)
