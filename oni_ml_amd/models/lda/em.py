"""Variational-EM LDA engine (replacement for the MPI oni-lda-c core).

Reference behaviour: oni-lda-c `lda est` (ml_ops.sh:80):
random/seeded/model init -> EM loop { zero ss; E-step over docs; M-step (lda_mle,
optional alpha Newton); conv = (L_old - L)/L_old; if conv < 0: VAR_MAX_ITER *= 2 }
while (conv < 0 or conv > EM_CONV or i <= 2) and i <= EM_MAX_ITER.

MI355X design:
* the corpus (CSR + CSC) and the model (word-major beta, fp64 like lda-c) stay resident in
  HBM for the whole run; one EM iteration = length-bucketed fp64 block Gauss-Seidel E-step
  kernels (csrc/hip/lda_gs64.hip, on 4 HIP streams so the long-document buckets overlap
  the short ones) -> deterministic CSC sufficient statistics -> (RCCL sparse row exchange
  or all-reduce when data-parallel) -> M-step + alpha Newton + the EM convergence test, all
  on the device and replayed as hipGraphs: the host reads the per-iteration history back once
  per batch of iterations.
* backends ("auto": hip on a GPU with the kernels, else cpu):
  "hip"   the gfx950 kernels (the MI355X engine);
  "cpu"   lda-c semantics in C++ (csrc/native/lda_ref.cpp: per-word Gauss-Seidel, or the GPU's block
          schedule with settings.gs_updates), multithreaded -- the engine of a GPU-less host;
  "torch" a vectorised Jacobi fixed point in torch (any device), a test rehearsal engine only: it is
          the one whose multi-rank statistics fold bitwise like one process
          (ONI_DIST_DETERMINISTIC=chain, tests/test_sharded_pipeline.py) and must be asked for by name.
"""
from __future__ import annotations

import math
import os
import threading
import time
import weakref
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np
import torch

from ... import knobs
from ...corpus.csr import Corpus, DeviceCorpus
from ...utils.trace import range_push, range_pop
from . import special
from .settings import LDASettings, LOG_FLOOR, NUM_INIT


@dataclass
class EMIterStats:
    iteration: int
    likelihood: float
    converged: float
    alpha: float
    seconds: float
    var_iter_mean: float
    var_iter_max: int
    var_max_iter: int


@dataclass
class LDAResult:
    log_beta: np.ndarray            # [K, V] float64 (lda-c .beta content)
    gamma: np.ndarray               # [D, K] float64 (lda-c .gamma content)
    alpha: float
    num_topics: int
    num_terms: int
    likelihoods: List[tuple] = field(default_factory=list)   # (L, conv) per EM iteration
    stats: List[EMIterStats] = field(default_factory=list)
    em_iterations: int = 0
    seconds: float = 0.0


def cphi_window_bounds(doc_ptr, budget_rows: int):
    """Contiguous nnz-balanced document windows of <= budget_rows corpus entries each (a document
    longer than the budget gets a window of its own): [{d0, d1, e0, e1}] covering every document."""
    from ...parallel.dist import shard_bounds
    ptr = np.asarray(doc_ptr, np.int64)
    nnz = int(ptr[-1])
    n0 = max(1, -(-nnz // max(1, int(budget_rows))))
    for B in range(n0, 4 * n0 + 1):
        cuts = [(a, b) for a, b in shard_bounds(ptr, B) if b > a]
        if max(int(ptr[b] - ptr[a]) for a, b in cuts) <= budget_rows:
            break
    else:
        # nnz-balanced cuts cannot isolate the over-long documents: greedy, one document at a time
        cuts, a = [], 0
        while a < len(ptr) - 1:
            b = a + 1
            while b < len(ptr) - 1 and ptr[b + 1] - ptr[a] <= budget_rows:
                b += 1
            cuts.append((a, b))
            a = b
    return [dict(d0=int(a), d1=int(b), e0=int(ptr[a]), e1=int(ptr[b])) for a, b in cuts]


def _cpu_threads() -> int:
    """Threads of the C++ lda-c engine (its result does not depend on the count)."""
    return knobs.threads(8)

def _hbm_total(device) -> int:
    """The device's HBM bytes from hipMemGetInfo.  (torch.cuda.get_device_properties first counts the
    devices through amd-smi: 0.11 s of a cold ml_ops process, profiles/r4_cold_start.md.)"""
    return int(torch.cuda.mem_get_info(device)[1])


def _stage_budget_gb(v: str) -> float:
    """ONI_GS_STAGE: the staged-rows budget in GB.  Until round 5 it was an on/off flag (1 = staged,
    4 GB cap): a value in (0, 1] is read as that flag, with a warning."""
    gb = float(v)
    if 0 < gb <= 1:
        import warnings
        warnings.warn(f"ONI_GS_STAGE={v}: read as the old on/off flag (4 GB budget); give the budget in GB > 1",
                      stacklevel=3)
        return 4.0
    return gb



class PinnedPool:
    """Pinned host buffers of the LAG saves' deferred device-to-host copies, reused once the file writer has
    let go of them.  A fresh process pins ~1.1 ms per 10 MB (profiles/r6q_pinned_probe.log); the headline
    day's six LAG saves (log beta, gamma, the checkpoint's class_word) took a new ~40 MB set each, ~42 ms of
    a cold ml_ops lda stage.  ``take`` returns a (tensor, ndarray) pair; when the ndarray and every view of
    it are gone (the writer's jobs finished), the tensor goes back to the free list of its shape."""

    def __init__(self, alloc: Optional[Callable] = None):
        self._free = {}
        self._lock = threading.Lock()
        self._alloc = alloc or (lambda shape, dtype: torch.empty(shape, dtype=dtype, pin_memory=True))
        self.allocated = 0           # buffers pinned so far (tests, records)

    def take(self, shape, dtype):
        key = (tuple(int(x) for x in shape), dtype)
        with self._lock:
            lst = self._free.get(key)
            t = lst.pop() if lst else None
        if t is None:
            t = self._alloc(key[0], dtype)
            self.allocated += 1
        arr = t.numpy()
        weakref.finalize(arr, self._give, key, t)
        return t, arr

    def _give(self, key, t):
        with self._lock:
            self._free.setdefault(key, []).append(t)


_PINNED = PinnedPool()


class DeviceHandoff:
    """A device tensor of a LAG save handed to a file-writer thread.  The thread driving the GPU only queues a
    device copy of the saved state and records ``event``; the writer's first ``get()`` copies the tensor to a
    pooled pinned host buffer on a side stream of its own (behind ``event``), waits for that stream only, and
    drops the device tensor.  The host buffers are then pinned and taken by the writer when it is ready to
    format, not by the EM loop at every save (profiles/r6_lda_stage.md)."""
    _streams = {}
    _slock = threading.Lock()

    def __init__(self, t: torch.Tensor, event):
        self._t, self._ev = t, event
        self.shape, self.dtype = tuple(t.shape), t.dtype
        self._lock = threading.Lock()
        self._host = None

    @classmethod
    def _stream(cls, device):
        with cls._slock:
            s = cls._streams.get(device)
            if s is None:
                s = cls._streams[device] = torch.cuda.Stream(device=device)
            return s

    def get(self) -> np.ndarray:
        with self._lock:
            if self._host is None:
                t = self._t
                s = self._stream(t.device)
                s.wait_event(self._ev)
                h, arr = _PINNED.take(self.shape, self.dtype)
                with torch.cuda.stream(s):
                    h.copy_(t, non_blocking=True)
                s.synchronize()
                self._host, self._t = arr, None
            return self._host


class LDAEngine:
    def __init__(self, corpus: Corpus, num_topics: int, settings: Optional[LDASettings] = None,
                 alpha_init: float = 2.5, backend: str = "auto", device=None, dist=None, seed: int = 0,
                 streams: int = 4, local_shard: bool = False, split_docs: bool = True,
                 split_min: Optional[int] = 4096, use_graph: bool = True, precision: str = "fp64",
                 emulate_shards: int = 0, doc_offset: int = 0, cphi_gb: Optional[float] = None,
                 suff_split: str = "auto", xsplit: Optional[dict] = None):
        """precision: "fp64" (the only engine: lda-c's double arithmetic; the hip backend runs the block
        Gauss-Seidel schedule of lda_gs64.hip).
        emulate_shards (torch backend, one process): reduce the sufficient statistics as the N
        document shards of ``dist.engine_bounds`` summed in shard order -- bitwise the N-rank run under
        ONI_DIST_DETERMINISTIC=1 (parallel/dist.py).
        local_shard: ``corpus`` is already this rank's shard; ``doc_offset`` its first global document
        (the row-sharded pipeline, corpus/sharded.py).
        cphi_gb (fp64 hip engine): HBM budget of the per-entry c.phi rows (nnz x KS x 8 bytes); a
        corpus whose rows exceed it runs its E-step in contiguous document windows, each followed by
        its share of the sufficient statistics (``_cphi_windows``).  None: ONI_CPHI_GB, else windows
        only when the rows would take more than 35 % of the GPU's memory.
        suff_split (fp64 hip engine): "auto" -- the longest-document bucket's entries reduced after it, the
        others while it still runs (``_build_suff_split``) when that overlaps anything; "off"; "force"."""
        self.cphi_gb = cphi_gb
        if suff_split not in ("auto", "off", "force"):
            raise ValueError(f"suff_split must be auto | off | force, got {suff_split!r}")
        self.suff_split = suff_split
        self.n_streams = max(2, int(streams))     # the E-step buckets' streams, the current one included
        self.xsplit = xsplit          # experimental XCD-split plan of the longest documents (ops/hip.py GSPlan)
        # the fused EM iteration's M-step launch refills the next E-step's staged rows (one rank); False: a
        # gs_stage launch before every E-step (tests/test_gs64.py pins the two bitwise equal)
        self.stage_fuse = True
        self.settings = settings or LDASettings()
        self.emulate_shards = int(emulate_shards)
        # cpu backend: lda-c's MPI ranks (document shards reduced in shard order; 1 = one process)
        self.cpu_shards = 1
        if precision != "fp64":
            raise ValueError(f"precision must be fp64 (lda-c's arithmetic), got {precision!r}")
        self.precision = precision
        self.K = int(num_topics)
        self.V = corpus.num_terms
        self.alpha = float(alpha_init)
        self.alpha_init = float(alpha_init)
        self.dist = dist
        self.seed = seed
        self.var_max_iter = self.settings.var_max_iter
        self.collect_iter_stats = False
        self.max_batch = 8          # EM iterations enqueued per host read-back (run())
        # run() without saves: batches of 4 -- the rest of the converging batch and the batch queued behind it
        # run as gated no-ops (to convergence on the headline day 51.33 -> 50.89 ms median of 7 against 8;
        # 2: 50.97, 1: 52.03; profiles/r6ar_converge_batch_ab.log)
        self.pipe_batch = 4
        if backend == "auto":
            from ...ops import hip as H
            if H.available():
                backend = "hip"
            elif torch.cuda.is_available():
                # a GPU without the kernels is a broken install, not a reason to run 2500x slower
                H.lib()
                raise RuntimeError("HIP extension loaded but unusable on this GPU")
            else:
                # a GPU-less host runs lda-c's own algorithm (C++, threads), never the Jacobi rehearsal engine
                backend = "cpu"
        self.backend = backend
        # ONI_DIST_DETERMINISTIC=chain (torch backend): sufficient statistics and the likelihood /
        # alpha_ss sums continue one sequential fold over the documents in corpus order, rank after
        # rank (parallel/shardio.chain): the model is bitwise the same for any number of ranks
        self._chain = backend == "torch" and knobs.get("ONI_DIST_DETERMINISTIC", "0") == "chain"
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if (
                backend == "hip" or torch.cuda.is_available()) and torch.cuda.is_available() else torch.device("cpu")
        self.device = torch.device(device)
        # shard (data parallel over documents)
        self.global_docs = corpus.num_docs
        if local_shard:
            # caller already hands this rank its own shard (weak-scaling bench, sharded pipeline)
            self.doc_range = (int(doc_offset), int(doc_offset) + corpus.num_docs)
            if dist is not None:
                self.global_docs = dist.allreduce_int(corpus.num_docs)
        elif dist is not None and dist.active:
            d0, d1 = dist.shard_range(corpus, self.K)
            self.doc_range = (d0, d1)
            corpus = corpus.slice_docs(d0, d1)
        else:
            self.doc_range = (0, corpus.num_docs)
        self.corpus = corpus
        self.D = corpus.num_docs
        self.fp64 = backend == "hip"
        self.use_graph = use_graph
        if self.fp64:
            self._init_gs64(corpus)
        elif backend == "torch":
            dev = self.device
            self.KS = self.K
            self.t_doc_ptr = torch.from_numpy(corpus.doc_ptr).to(dev)
            self.t_word = torch.from_numpy(corpus.word_idx.astype(np.int64)).to(dev)
            self.t_cnt = torch.from_numpy(corpus.counts.astype(np.float64)).to(dev)
            self.beta = torch.zeros(self.V, self.K, dtype=torch.float64, device=dev)
            self.cw = torch.zeros(self.V, self.K, dtype=torch.float64, device=dev)
            self.gamma = torch.zeros(self.D, self.K, dtype=torch.float64, device=dev)
        elif backend == "cpu":
            from ...ops import native
            self._native = native.lib()
            self.KS = self.K
            self.beta = torch.zeros(self.V, self.K, dtype=torch.float64)
            self.cw = torch.zeros(self.V, self.K, dtype=torch.float64)
            self.gamma = torch.zeros(self.D, self.K, dtype=torch.float64)
        else:
            raise ValueError(f"unknown backend {backend}")
        if backend != "hip":
            self.class_total = torch.zeros(self.KS, dtype=torch.float64, device=self.cw.device)
        self._xchg = self._make_exchange(corpus)
        # sparse exchange on the GPU: suff-stats of the shared words first, so their all-to-all runs
        # while the suff-stats of the rank's private words (the bulk) are computed
        self._overlap = self._xchg is not None and backend == "hip" and \
            knobs.get("ONI_DIST_EXCHANGE", "auto") != "sparse-serial" and getattr(self, "_cwin", None) is None
        if self._overlap:
            from ...ops import hip as H
            # only this rank's words: rows of other words stay zero in cw_local and are never read
            # (the E-step touches only local words; the M-step is restricted to them below)
            shared = np.unique(self._xchg.send_idx.cpu().numpy())
            local = self._xchg.local_ids.cpu().numpy()
            private = np.setdiff1d(local, shared, assume_unique=True)
            self._plan_a = H.SuffPlan(self.dc.word_len, self.device, words=shared)
            self._plan_b = H.SuffPlan(self.dc.word_len, self.device, words=private)
            # never below the rows _init_gs64 sized for the K > 32 per-stream groups (e_step()'s phase='all')
            nb = max(self._plan_a.n_blocks + self._plan_b.n_blocks, self.suff_plan.n_blocks, 1,
                     int(self._suff_part.shape[0]))
            self._suff_part = torch.zeros(nb, 2 + self.KS, dtype=torch.float64, device=self.device)
            self._graph_a = self._graph_b = None

    # ------------------------------------------------------------ metrics
    def _comm_begin(self):
        if self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ("cuda", ev)
        return ("host", time.perf_counter())

    def _comm_end(self, tok):
        if not hasattr(self, "_comm_events"):
            self._comm_events, self._comm_host_s, self._comm_iters = [], 0.0, 0
        self._comm_iters += 1
        if tok[0] == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._comm_events.append((tok[1], ev))
        else:
            self._comm_host_s += time.perf_counter() - tok[1]

    def comm_seconds(self) -> float:
        """Time of the cross-rank reductions so far (stream time from issue to the compute stream's
        wait on them; host time for CPU collectives)."""
        if not hasattr(self, "_comm_events"):
            return 0.0
        t = self._comm_host_s
        if self._comm_events:
            torch.cuda.synchronize(self.device)
            t += sum(a.elapsed_time(b) for a, b in self._comm_events) / 1e3
        return t

    def exchange_bytes_per_iteration(self) -> int:
        """Payload this rank hands to the collectives every EM iteration (class_word rows + scalars)."""
        if self.dist is None or not self.dist.active:
            return 0
        el = self.cw.element_size()
        scal = (2 + self.KS) * 8
        if self._xchg is not None:
            return int(self._xchg.rows * self._xchg.width * el + scal)
        return int(self.cw.numel() * el + scal)

    def metrics(self, seconds: Optional[float] = None, em_iterations: Optional[int] = None) -> dict:
        """Run metrics for metrics.jsonl / lda_stats.json: peak HBM, exchange payload and
        time per EM iteration, the variational-iteration histogram of the last E-step, docs/s."""
        it = self.iters.cpu().numpy() if isinstance(self.iters, torch.Tensor) else np.asarray(self.iters)
        hist = np.bincount(it.astype(np.int64)).tolist() if it.size else []
        out = dict(schedule=self.schedule, exchange=self.exchange_mode,
                   exchange_bytes_per_iter=self.exchange_bytes_per_iteration(),
                   var_iter_hist=hist, var_iter_mean=float(it.mean()) if it.size else 0.0,
                   var_iter_max=int(it.max()) if it.size else 0)
        n = getattr(self, "_comm_iters", 0)
        out["exchange_seconds_per_iter"] = self.comm_seconds() / n if n else 0.0
        if self.device.type == "cuda":
            out["peak_hbm_bytes"] = int(torch.cuda.max_memory_allocated(self.device))
            out["hbm_total_bytes"] = _hbm_total(self.device)
        if seconds and em_iterations:
            out["docs_per_sec"] = self.global_docs * em_iterations / seconds
        return out

    @property
    def schedule(self) -> str:
        """Variational update schedule of this engine (bench / metrics records)."""
        if self.backend == "hip" and self.fp64:
            return f"block Gauss-Seidel, fp64, {self._U} gamma refreshes per sweep (lda-c per-word up to {self._U} words)"
        if self.backend == "cpu":
            u = resolved_gs_updates(self.settings, self.K)
            return "lda-c per-word Gauss-Seidel, fp64" if u == 0 else f"block Gauss-Seidel, fp64, {u} refreshes per sweep"
        return "Jacobi, fp64"

    # ------------------------------------------------- fp64 block Gauss-Seidel
    def gs_updates(self) -> int:
        """U: gamma refreshes per sweep of the fp64 engine (settings.gs_updates, 0 = the default 32,
        -1 = ``parity_gs_updates(K)``)."""
        from ...ops import hip as H
        KS = H.padded_topics(self.K)
        u = int(self.settings.gs_updates)
        if u < 0:
            u = parity_gs_updates(self.K)
        u = u or min(32, H.gs_umax(KS))
        if not 1 <= u <= H.gs_umax(KS):
            raise ValueError(f"gs_updates={u}: the GPU engine supports 1..{H.gs_umax(KS)} at K={self.K}")
        return u

    def _init_gs64(self, corpus: Corpus):
        """Buffers of the fp64 engine (csrc/hip/lda_gs64.hip): everything lda-c keeps in double is double
        here (beta, class_word, gamma, the per-entry c*phi rows, likelihood and alpha terms)."""
        from ...ops import hip as H
        self.KS = KS = H.padded_topics(self.K)
        self.dc = DeviceCorpus.build(corpus, self.device)
        dev, D, V, nnz = self.device, self.D, self.V, corpus.nnz
        self._U = self.gs_updates()
        f64 = torch.float64
        self._cwin = self._cphi_windows(corpus, KS)
        if self._cwin is None:
            self.gs_plan = H.GSPlan(self.dc.doc_len, KS, self._U, dev, xsplit=self.xsplit)
            self._split_sums(self.gs_plan, corpus)
            rows = nnz
        else:
            self.gs_plan = None
            for w in self._cwin:
                w["gp"] = H.GSPlan(self.dc.doc_len, KS, self._U, dev, doc_range=(w["d0"], w["d1"]))
                self._split_sums(w["gp"], corpus)
            rows = max(w["e1"] - w["e0"] for w in self._cwin)
        # one zero pad row past the vocabulary: gs_smallw's constant-offset row loads may read past row V - 1
        self.beta = torch.zeros(V + 1, KS, dtype=f64, device=dev)[:V]
        self._stages = self._build_stages(corpus, KS)
        self.cw = torch.zeros(V, KS, dtype=f64, device=dev)
        self.gamma = torch.zeros(D, KS, dtype=f64, device=dev)
        # one pad row past the last entry: the suff-stats kernel's paired row loads (KS > 32) may read into it
        self.cphi = torch.zeros(rows + 1, KS, dtype=f64, device=dev)[:rows]
        self.lik = torch.zeros(D, dtype=f64, device=dev)
        self.ass = torch.zeros(D, dtype=f64, device=dev)
        self.iters = torch.zeros(D, dtype=torch.int32, device=dev)
        # (high-priority side streams for the longest-document buckets measured slower: 2.13 -> 2.40 ms
        # per EM iteration at K = 20, 3.33 -> 3.84 at K = 50; profiles/r3_tuning_log.md)
        self._streams = [torch.cuda.Stream(device=dev) for _ in range(max(1, self.n_streams - 1))]
        self._red = torch.zeros(2 + KS, dtype=f64, device=dev)
        self._scalars = self._red[:2]
        self.class_total = self._red[2:]
        self._distributed = self.dist is not None and self.dist.active
        self._cw_local = torch.zeros_like(self.cw) if self._distributed else self.cw
        self._red_local = torch.zeros_like(self._red) if self._distributed else self._red
        self.suff_plan = H.SuffPlan(self.dc.word_len, dev)
        self._suff_part = torch.zeros(max(self.suff_plan.n_blocks, 1), 2 + KS, dtype=f64, device=dev)
        self._done_count = torch.zeros(1, dtype=torch.int32, device=dev)
        self._alpha_dummy = torch.zeros(1, dtype=f64, device=dev)
        self._ct_fresh = False
        self._params = torch.zeros(H.PARAM_COUNT, dtype=f64, device=dev)
        self._gate = self._params[H.PARAM_DONE:H.PARAM_DONE + 1]
        self._hist_cap = 64
        self._ctlhist = torch.zeros(8 + H.HIST_COLS * self._hist_cap, dtype=f64, device=dev)
        self._ctl, self._hist = self._ctlhist[:8], self._ctlhist[8:]
        self._ev_fork = torch.cuda.Event()
        self._ev_join = [torch.cuda.Event() for _ in range(len(self._streams) + 1)]
        self._graph = None
        self._mgraph, self._mgraph_key = None, None
        self._fgraphs, self._fgraph_key = {}, None
        self._out_host = torch.zeros(self._ctlhist.numel(), dtype=f64).pin_memory()
        self._pushed = None
        self._suff_split = None
        if self._cwin is not None:
            self._build_window_suff()
        elif self.suff_split != "off":
            self._suff_split = self._build_suff_split()

    @staticmethod
    def _split_sums(gp, corpus: Corpus) -> None:
        """The split batches' chunk count sums, once per plan (ops/hip.py GSSplitPlan.chunk_sums)."""
        from ...ops import hip as H
        if isinstance(gp.split, H.GSSplitPlan):
            gp.split.chunk_sums(corpus.doc_ptr, corpus.counts)

    def _build_stages(self, corpus: Corpus, KS: int) -> dict:
        """Staged beta rows (ops/hip.py GSStage) of every kGsTeam8 launch at KS <= 32, keyed by the id of
        the launch's order tensor.  ONI_GS_STAGE = the budget in GB (default 4; 0 turns them off): a plan
        whose copies would exceed it is left unstaged."""
        from ...ops import hip as H
        gb = _stage_budget_gb(knobs.get("ONI_GS_STAGE", "4"))
        if KS > 32 or gb <= 0 or self._U > 32:   # U > 32: the topic-group team reads beta (no gs_wsteam)
            return {}
        cap = gb * 2**30
        plans = [self.gs_plan] if self._cwin is None else [w["gp"] for w in self._cwin]
        out = {}
        for gp in plans:
            for var, order in gp.plan:
                if var != H.GS_TEAM8:
                    continue
                o = order.cpu().numpy()
                o = o[o >= 0]
                # GSStage pads every document to whole 64-row tiles
                need = int((-(-(corpus.doc_ptr[o + 1] - corpus.doc_ptr[o]) // 64)).sum()) * 64 * KS * 8
                if need > cap:
                    continue
                cap -= need
                out[id(order)] = H.GSStage(order, corpus.doc_ptr, KS, self.device)
        return out

    def _cphi_windows(self, corpus: Corpus, KS: int):
        """Contiguous document windows [d0, d1) of <= the c.phi budget's rows each (nnz-balanced, a
        document longer than the budget alone in its window), or None when the whole corpus fits.

        The E-step of a window writes its c.phi rows into one shared buffer, the window's slice of the
        sufficient statistics (a CSC subset) adds them to class_word (in place, window order), then the
        next window runs: peak HBM drops from nnz x KS x 8 bytes to the largest window's rows, for one
        more suff-stats pass per window.  class_word[w] is summed window by window, so it differs from
        the one-buffer engine in the last bits (sums in another order); fixed for a given budget."""
        nnz = corpus.nnz
        row_bytes = KS * 8
        gb = self.cphi_gb
        if gb is None and knobs.get("ONI_CPHI_GB"):
            gb = float(knobs.get("ONI_CPHI_GB"))
        if gb is None:
            total = _hbm_total(self.device) if self.device.type == "cuda" else 0
            if not total or nnz * row_bytes <= 0.35 * total:
                return None
            gb = 0.25 * total / 2**30
        budget = max(1, int(gb * 2**30) // row_bytes)
        if gb <= 0 or budget >= nnz:
            return None
        return cphi_window_bounds(corpus.doc_ptr, budget)

    def _build_window_suff(self):
        """Per window: its CSC subset (entry ids relative to the window's first entry) and a suff plan
        over only the words it holds (the other rows of class_word are not touched by its pass); plus
        the closing pass over the whole vocabulary with no entries, which yields the class totals and
        the likelihood / alpha_ss slices (``_launch_windows``)."""
        from ...ops import hip as H
        dc, dev, V = self.dc, self.device, self.V
        wlen = (dc.word_ptr[1:] - dc.word_ptr[:-1]).long()
        word_of = torch.repeat_interleave(torch.arange(V, device=dev), wlen)      # once for all windows
        need = 1
        for w in self._cwin:
            keep = (dc.csc_doc >= w["d0"]) & (dc.csc_doc < w["d1"])
            cnt = torch.bincount(word_of[keep], minlength=V)
            ptr = torch.zeros(V + 1, dtype=torch.int64, device=dev)
            ptr[1:] = torch.cumsum(cnt, 0)
            w["wp"] = ptr.to(torch.int32)
            w["ce"] = (dc.csc_ent[keep] - w["e0"]).contiguous()
            wl = cnt.cpu().numpy()
            w["sp"] = H.SuffPlan(wl, dev, words=np.flatnonzero(wl))
            need = max(need, w["sp"].n_blocks)
        del word_of
        self._win_total = dict(wp=torch.zeros(V + 1, dtype=torch.int32, device=dev),
                               ce=torch.zeros(1, dtype=torch.int32, device=dev),
                               sp=H.SuffPlan(np.zeros(V, np.int64), dev))
        need = max(need, self._win_total["sp"].n_blocks)
        if self._suff_part.shape[0] < need:
            self._suff_part = torch.zeros(need, self._suff_part.shape[1], dtype=torch.float64, device=dev)

    def _build_suff_split(self):
        """Early / late sufficient statistics: class_word[w] = (sum over w's entries in documents of the
        other buckets, computed while the longest-document bucket still runs) + (sum over its entries in
        the longest-document bucket, after it).  Two CSC subsets of the corpus; the late pass adds the
        early rows first (``gs_suff64(base=...)``), so the order is fixed.  None when there is nothing
        to overlap (one bucket, or the late bucket holds most of the entries)."""
        from ...ops import hip as H
        gp, dc, dev = self.gs_plan, self.dc, self.device
        if len(gp.plan) + (gp.split is not None) < 2:
            return None
        if gp.KS > 32:
            return self._build_suff_groups()
        key = self._late_key(gp)
        if key == "split":
            late = np.asarray(sorted(gp.split.segments), np.int64)
        else:
            o = gp.plan[key][1].cpu().numpy()
            late = o[o >= 0].astype(np.int64)
        force = self.suff_split == "force"
        if late.size == 0 or (not force and dc.doc_len[late].sum() > 0.6 * max(1, int(dc.doc_len.sum()))):
            return None
        mask = torch.zeros(self.D, dtype=torch.bool, device=dev)
        mask[torch.from_numpy(late).to(dev)] = True
        wpE, ceE, lenE = H.csc_subset(dc.word_ptr, dc.csc_ent, dc.csc_doc, ~mask)
        wpL, ceL, lenL = H.csc_subset(dc.word_ptr, dc.csc_ent, dc.csc_doc, mask)
        planE, planL = H.SuffPlan(lenE, dev), H.SuffPlan(lenL, dev)
        need = max(planE.n_blocks, planL.n_blocks, 1)
        if self._suff_part.shape[0] < need:
            self._suff_part = torch.zeros(need, self._suff_part.shape[1], dtype=torch.float64, device=dev)
        return dict(wpE=wpE, ceE=ceE, planE=planE, wpL=wpL, ceL=ceL, planL=planL,
                    cw_early=torch.zeros_like(self.cw), late_docs=int(late.size))

    def _stream_slots(self, gp, late: bool) -> list:
        """Stream of every work item ([split] + gp.plan) as _launch_buckets dispatches them: 0 = the current
        stream, i >= 1 = self._streams[i - 1].  late: the _late_key bucket alone on stream 1, the others
        round-robin over the remaining side streams and then the current stream."""
        n = len(gp.plan) + (gp.split is not None)
        key = self._late_key(gp)
        late_i = 0 if key == "split" else key + (gp.split is not None)
        others = [i for i in range(1, len(self._streams) + 1) if not (late and i == 1)] + [0]
        out, oi = [], 0
        for si in range(n):
            if late and si == late_i:
                out.append(1)
            else:
                out.append(others[oi % len(others)])
                oi += 1
        return out

    def _build_suff_groups(self):
        """Per-stream sufficient statistics (KS > 32): each stream's suff-stats pass runs on that stream as
        soon as its own buckets are done, so only the last-finishing stream's pass (and a short combine)
        follows the E-step, whichever stream that is (the K = 100 shard: the 8-wave team; 100 M events:
        the tiny bucket, which waits behind the split documents: 18.5 ms of suff-stats after the E-step,
        profiles/r5y_100m/timeline.txt).

        A word whose entries all lie in one stream's documents gets its class_word row from that stream's
        pass directly; the other words' per-stream rows go to a scratch (compact CSC per stream) and the
        combine pass -- one more gs_suff64 over a CSC of scratch rows in stream order -- sums them.  The
        sum order is fixed by the plan, never by which stream finishes first: bitwise reproducible.
        class_total's partial rows come from the direct rows and the combine only."""
        import numpy as np
        from ...ops import hip as H
        gp, dc, dev = self.gs_plan, self.dc, self.device
        slots = self._stream_slots(gp, late=True)
        work_docs = []
        if gp.split is not None:
            work_docs.append(np.asarray(sorted(gp.split.segments), np.int64))
        for _, order in gp.plan:
            o = order.cpu().numpy()
            work_docs.append(o[o >= 0].astype(np.int64))
        keys = sorted(set(slots))
        if len(keys) < 2:
            return None
        V = self.V
        groups, lens = [], []
        for k in keys:
            docs = np.concatenate([d for d, sl in zip(work_docs, slots) if sl == k])
            mask = torch.zeros(self.D, dtype=torch.bool, device=dev)
            mask[torch.from_numpy(docs).to(dev)] = True
            wp, ce, ln = H.csc_subset(dc.word_ptr, dc.csc_ent, dc.csc_doc, mask)
            groups.append(dict(slot=k, wp=wp, ce=ce))
            lens.append(ln.astype(np.int64))
        gpl = H.suff_group_plan(lens, V)
        if gpl is None:
            return None                                  # no word shared between streams: nothing to combine
        for g, ln, u, mw, off in zip(groups, lens, gpl["unique"], gpl["multi"], gpl["off"]):
            g["plan_u"] = H.SuffPlan(ln, dev, words=u) if u.size else None
            g["m"], g["off"], g["plan_m"] = int(mw.size), off, None
            if mw.size:
                g["wp_m"], g["ce_m"] = H.csc_compact(g["wp"], g["ce"], mw)
                g["plan_m"] = H.SuffPlan(ln[mw], dev)
        rows_off = gpl["rows"]
        comb = dict(wp=torch.from_numpy(gpl["wp"].astype(np.int32)).to(dev),
                    ce=torch.from_numpy(gpl["ce"].astype(np.int32)).to(dev),
                    plan=H.SuffPlan(gpl["cnt"], dev, words=gpl["shared"]))
        # scratch rows of the shared words, one pad row past the last (KS > 32 row loads)
        xs = torch.zeros(rows_off + 1, self.KS, dtype=torch.float64, device=dev)[:rows_off]
        # partial rows: [direct passes | combine] are summed into class_total; the scratch passes' after them
        nb = 0
        for g in groups:
            g["pu0"] = nb
            nb += g["plan_u"].n_blocks if g["plan_u"] is not None else 0
        comb["p0"] = nb
        nsum = nb + comb["plan"].n_blocks
        nb = nsum
        for g in groups:
            g["pm0"] = nb
            nb += g["plan_m"].n_blocks if g["plan_m"] is not None else 0
        if self._suff_part.shape[0] < nb:
            self._suff_part = torch.zeros(nb, self._suff_part.shape[1], dtype=torch.float64, device=dev)
        return dict(mode="groups", groups=groups, comb=comb, xs=xs, n_sum=nsum)

    def _suff_group_passes(self, g, ss):
        """One stream's suff-stats passes (on the current stream): its direct rows, then its shared words'
        rows into the scratch."""
        from ...ops import hip as H
        gate, part = self._gate, self._suff_part
        if g["plan_u"] is not None:
            H.gs_suff64(g["wp"], g["ce"], g["plan_u"], self.cphi, self._cw_local,
                        part[g["pu0"]:g["pu0"] + max(g["plan_u"].n_blocks, 1)], gate=gate)
        if g["plan_m"] is not None:
            H.gs_suff64(g["wp_m"], g["ce_m"], g["plan_m"], self.cphi, ss["xs"][g["off"]:g["off"] + g["m"]],
                        part[g["pm0"]:g["pm0"] + max(g["plan_m"].n_blocks, 1)], gate=gate)

    @staticmethod
    def _late_key(gp):
        """The bucket the late suff-stats pass waits for (it runs alone on streams[1]; the early pass covers
        every other bucket's words): the one expected to finish last.  At K > 32 that is the 8-wave team
        when there is one -- the split documents (dispatched first, co-resident) finished at 9.9 ms of a
        30.6 ms K = 100 iteration and the 8-wave team last, so with the split as the late bucket both passes
        ran after everything (profiles/r5q_k100_timeline.txt) -- else the split, else plan[0] (the
        longest-document bucket at K <= 32)."""
        from ...ops import hip as H
        if gp.KS > 32:
            for want in (H.GS_TEAM8, H.GS_TEAM4):
                for i, (var, _) in enumerate(gp.plan):
                    if var == want:
                        return i
        return "split" if gp.split is not None else 0

    def _launch_estep64(self, newton_key=None, phase: str = "all"):
        """fp64 E-step: length buckets on 4 streams (longest first), one join, then the CSC
        suff-stats (+ likelihood / alpha_ss slices), one column pass, [M-step + Newton + control]."""
        from ...ops import hip as H
        dc, prm, gate = self.dc, self._params, self._gate
        main = torch.cuda.current_stream(self.device)
        if phase == "B":
            pa, pb = self._plan_a, self._plan_b
            # the likelihood / alpha_ss slices ride on phase A's launch unless it has no workgroups
            # (a rank that shares no word with any other)
            H.gs_suff64(dc.word_ptr, dc.csc_ent, pb, self.cphi, self._cw_local,
                        self._suff_part[pa.n_blocks:pa.n_blocks + pb.n_blocks], gate=gate,
                        scalars=None if pa.n_blocks else (self.lik, self.ass, 0, self.lik.numel()))
            H.colsum_partials(self._suff_part, pa.n_blocks + pb.n_blocks, self._red_local, gate=gate)
            self._red.copy_(self._red_local)
            return
        if self._cwin is not None:
            self._launch_windows(newton_key, phase)
            return
        gp = self.gs_plan
        # early / late suff-stats (phase "all"): work[0], the longest-document bucket, runs alone on
        # streams[1] (late_s); the early pass joins every other stream
        ss = self._suff_split if (phase == "all" and len(gp.plan) + (gp.split is not None) >= 2) else None
        # one rank, fused EM iteration: this launch's M-step refills the staged rows for the next E-step,
        # and this E-step uses the rows the previous M-step (or the batch's opening refill) left
        fused = newton_key is not None and phase == "all" and bool(self._fused_stages(gp))
        grp = ss if (ss is not None and ss.get("mode") == "groups" and phase == "all") else None
        used, late_s = self._launch_buckets(gp, ss is not None, fused_stage=fused, groups=grp)
        if phase == "estep":             # the document kernels only (final inference pass)
            return
        scal = (self.lik, self.ass, 0, self.lik.numel())
        if grp is not None:
            c = grp["comb"]
            H.gs_suff64(c["wp"], c["ce"], c["plan"], grp["xs"], self._cw_local,
                        self._suff_part[c["p0"]:c["p0"] + max(c["plan"].n_blocks, 1)], gate=gate, scalars=scal)
            H.colsum_partials(self._suff_part, grp["n_sum"], self._red_local, gate=gate)
            self._finish_suff64(newton_key, stages=self._fused_stages(gp) if fused else ())
            return
        if late_s is not None:
            H.gs_suff64(ss["wpE"], ss["ceE"], ss["planE"], self.cphi, ss["cw_early"], self._suff_part, gate=gate)
            main.wait_event(self._ev_join[used.index(late_s)])
            H.gs_suff64(ss["wpL"], ss["ceL"], ss["planL"], self.cphi, self._cw_local, self._suff_part, gate=gate,
                        scalars=scal, base=ss["cw_early"])
            H.colsum_partials(self._suff_part, ss["planL"].n_blocks, self._red_local, gate=gate)
            self._finish_suff64(newton_key, stages=self._fused_stages(gp) if fused else ())
            return
        if phase == "A":
            H.gs_suff64(dc.word_ptr, dc.csc_ent, self._plan_a, self.cphi, self._cw_local,
                        self._suff_part[:max(self._plan_a.n_blocks, 1)], gate=gate, scalars=scal)
            self._xchg.pack(self._cw_local)
            return
        sp = self.suff_plan
        H.gs_suff64(dc.word_ptr, dc.csc_ent, sp, self.cphi, self._cw_local, self._suff_part[:max(sp.n_blocks, 1)],
                    gate=gate, scalars=scal)
        H.colsum_partials(self._suff_part, sp.n_blocks, self._red_local, gate=gate)
        self._finish_suff64(newton_key, stages=self._fused_stages(gp) if fused else ())

    def _fused_stages(self, gp) -> list:
        """The staged-row sets of plan ``gp`` that the fused M-step launch refills (one rank, staged rows
        refilled on the main stream, at most 2 sets; ``stage_fuse = False``: none, a gs_stage launch
        before every E-step as before)."""
        if self._distributed or self._cwin is not None or not self.stage_fuse:
            return []
        sts = [self._stages[id(order)] for _, order in gp.plan if id(order) in self._stages]
        return sts if len(sts) <= 2 else []

    def _refill_stages(self):
        """gs_stage for every staged set of the plan (before a batch of fused EM iterations: beta may
        have been set by the host since the last fused M-step)."""
        from ...ops import hip as H
        for st in self._fused_stages(self.gs_plan):
            H.gs_stage(self.beta, self.dc.word_idx, st, gate=self._gate)

    def _launch_buckets(self, gp, late: bool = False, win=None, fused_stage: bool = False, groups=None):
        """The document kernels of GSPlan ``gp`` on 4 streams, joined back into the current stream.
        late: work[0] (the longest-document bucket) stays un-joined on streams[1], returned as late_s,
        for the early / late suff-stats; win: one of the c.phi windows (``_cphi_windows``) -- the document
        kernels write its entries into the first rows of the shared buffer."""
        from ...ops import hip as H
        dc, prm = self.dc, self._params
        main = torch.cuda.current_stream(self.device)
        streams = [main] + self._streams
        # staged rows refilled before the fork: the team8 launch is then the first dispatched, instead of
        # queueing behind the other buckets' workgroups for whole CUs (1.861 vs 1.904-1.933 ms per EM
        # iteration refilled on the bucket's own stream; profiles/r3_tuning_log.md)
        if not fused_stage:                     # fused: the previous M-step launch refilled them
            for var, order in gp.plan:
                st = self._stages.get(id(order))
                if st is not None:
                    H.gs_stage(self.beta, dc.word_idx, st, gate=self._gate)
        self._ev_fork.record(main)
        used = []
        # side streams: the long-document buckets (critical path) are dispatched first, the split
        # documents' batches (back to back on one stream) before everything
        work = list(gp.plan)
        if gp.split is not None:
            work.insert(0, ("split", gp.split.batches))
        # the late bucket (_late_key) runs alone on late_s = streams[1]: no other bucket may share it (the
        # early pass would read their cphi rows before they are written); the others round-robin over the
        # remaining streams in dispatch order
        # groups (the per-stream suff-stats, _build_suff_groups): every stream is joined after its passes
        late_s = streams[1] if (late and groups is None) else None
        # (the tiny bucket, last, follows the split / first side-stream bucket instead of queueing behind the
        # 16-lane bucket on the main stream: K = 100 shard 29.4 -> see r5u)
        slots = self._stream_slots(gp, late)
        # a c.phi window: the buffer's first e1 - e0 rows hold the window's entries
        cphi = self.cphi if win is None else self.cphi[:win["e1"] - win["e0"]]
        ent_base = None if win is None else win["e0"]
        for si, (var, order) in zip(range(len(work)), work):
            s = streams[slots[si]]
            if s is not main and s not in used:
                s.wait_event(self._ev_fork)
                used.append(s)
            with torch.cuda.stream(s):
                if var == "split":
                    for batch in order:
                        launch = H.gs_xsplit if batch.get("x") else H.gs_split
                        launch(dc.doc_ptr, dc.word_idx, dc.counts, self.beta, self.K, self._U, prm, self.gamma,
                               cphi, self.lik, self.ass, self.iters, batch, ent_base=ent_base)
                else:
                    st = self._stages.get(id(order))
                    H.gs_estep(dc.doc_ptr, dc.word_idx, dc.counts, order, self.beta, self.K, self._U, prm,
                               self.gamma, cphi, self.lik, self.ass, self.iters, var, ent_base=ent_base, stage=st)
        if groups is not None:
            for g in groups["groups"]:
                with torch.cuda.stream(streams[g["slot"]]):
                    self._suff_group_passes(g, groups)
        # every bucket but work[0] is joined first and the early pass overlaps work[0]
        for j, s in enumerate(used):
            self._ev_join[j].record(s)
            if s is not late_s:
                main.wait_event(self._ev_join[j])
        return used, late_s

    def _launch_windows(self, newton_key, phase: str):
        """E-step in c.phi windows: per window its document kernels, then its CSC subset's rows added
        to class_word in place (window 0 writes, later windows add); the likelihood / alpha_ss slices
        and the class totals ride on the last window's pass."""
        from ...ops import hip as H
        if phase not in ("all",):
            raise NotImplementedError(f"c.phi windows: E-step phase {phase!r}")
        gate = self._gate
        scal = (self.lik, self.ass, 0, self.lik.numel())
        cw = self._cw_local
        cw.zero_()
        for w in self._cwin:
            self._launch_buckets(w["gp"], win=w)
            # only the window's words: their rows += the window's entries (in place)
            H.gs_suff64(w["wp"], w["ce"], w["sp"], self.cphi[:w["e1"] - w["e0"]], cw, self._suff_part, gate=gate,
                        base=cw)
        # closing pass, every word and no entries: rows unchanged, column sums + likelihood slices
        tp = self._win_total
        H.gs_suff64(tp["wp"], tp["ce"], tp["sp"], self.cphi[:1], cw, self._suff_part, gate=gate, scalars=scal,
                    base=cw)
        H.colsum_partials(self._suff_part, tp["sp"].n_blocks, self._red_local, gate=gate)
        self._finish_suff64(newton_key)

    def _finish_suff64(self, newton_key, stages=()):
        if self._distributed:
            if self._xchg is not None:
                self._xchg.pack(self._cw_local)
            else:
                self.cw.copy_(self._cw_local)
            self._red.copy_(self._red_local)
        if newton_key is not None:
            self._launch_beta_control(newton_key, stages)

    def _make_exchange(self, corpus: Corpus):
        """Sparse class_word exchange (parallel/dist.py VocabExchange) when the ranks' vocabularies
        overlap little; ONI_DIST_EXCHANGE = auto (default) | sparse | sparse-serial | dense.  Collective:
        every rank builds it (or none does)."""
        d = self.dist
        if d is None or not d.active or self.backend == "cpu" or self._chain:
            return None
        mode = knobs.get("ONI_DIST_EXCHANGE", "auto")
        if mode == "dense" or getattr(d, "deterministic", False):
            # deterministic mode: one ordered reduction of the whole matrix (parallel/dist.py)
            return None
        from ...parallel.dist import VocabExchange
        words = np.unique(corpus.word_idx) if corpus.nnz else np.zeros(0, np.int64)
        x = VocabExchange(d, words, self.V, self.KS, self.cw.device, self.cw.dtype)
        return x if (mode in ("sparse", "sparse-serial") or x.worthwhile()) else None

    @property
    def exchange_mode(self) -> str:
        if self.dist is None or not self.dist.active:
            return "none"
        return "sparse-alltoall" if self._xchg is not None else "dense-allreduce"

    def global_cw(self) -> torch.Tensor:
        """class_word summed over all ranks for every word (collective under the sparse exchange,
        where a rank only holds its own words' rows)."""
        if self._xchg is None:
            return self.cw
        return self._xchg.global_rows(self.cw)

    # ------------------------------------------------------------------ init
    def init_random(self, seed: Optional[int] = None):
        """random_initialize_ss + lda_mle(..., 0): cw[k][w] = 1/V + U(0,1).  U comes from a counter-based
        generator (splitmix64 of (seed, k V + w)): the fp64 HIP engine fills class_word on the device
        (no host stream, no 8-byte-per-entry upload), every other backend gets the same bits from the
        native ``random_ss``."""
        s = self.seed if seed is None else seed
        if self.backend == "hip" and self.fp64:
            from ...ops import hip as H
            H.init_random_ss(self.cw, self.K, s)
            H.colsum_partials(self.cw, self.V, self.class_total)
            self._mstep_beta()
        else:
            from ...ops import native
            self._set_ss_host(native.lib().random_ss(self.K, self.V, int(s) & 0xFFFFFFFFFFFFFFFF))
        self.alpha = self.alpha_init

    def init_seeded(self, corpus_global: Optional[Corpus] = None, seed: Optional[int] = None):
        """corpus_initialize_ss: NUM_INIT random docs per topic + 1 smoothing.  Every rank draws the
        same global document ids; a rank adds the words of the chosen documents it holds, and the
        integer counts are summed over the ranks (exact in any order).  ``corpus_global``: the whole
        corpus when every rank has it (then no reduction is needed)."""
        rng = np.random.default_rng(self.seed if seed is None else seed)
        local = corpus_global is None
        c = self.corpus if local else corpus_global
        d0 = self.doc_range[0] if local else 0
        D = self.global_docs if local else corpus_global.num_docs
        cw = np.zeros((self.K, self.V))
        for k in range(self.K):
            for _ in range(NUM_INIT):
                d = int(math.floor(rng.random() * D)) - d0
                if 0 <= d < c.num_docs:
                    a, b = c.doc_ptr[d], c.doc_ptr[d + 1]
                    np.add.at(cw[k], c.word_idx[a:b], c.counts[a:b])
        if local and self.dist is not None and self.dist.active:
            import torch.distributed as td
            t = torch.from_numpy(cw).to(self.dist._coll_device())
            td.all_reduce(t)
            cw = t.cpu().numpy()
        cw += 1.0
        self._set_ss_host(cw)
        self.alpha = self.alpha_init

    def init_from_model(self, log_beta: np.ndarray, alpha: float):
        """Resume path (lda-c `load_lda_model`): beta from log p(w|z)."""
        lb = np.asarray(log_beta, dtype=np.float64)
        if lb.shape != (self.K, self.V):
            raise ValueError(f"model shape {lb.shape} != ({self.K}, {self.V})")
        cw = np.exp(lb)
        self._set_ss_host(cw, normalized=True)
        self.alpha = float(alpha)

    def state_arrays(self) -> dict:
        """Exact engine state (sufficient statistics in the engine's own precision) for checkpoints."""
        # copy=True: host arrays never alias live engine buffers (CPU backend), since files are written
        # by a background thread while EM continues
        return dict(cw=self.global_cw().to("cpu", copy=True).numpy(),
                    class_total=self.class_total.to("cpu", copy=True).numpy())

    def load_state_arrays(self, cw: np.ndarray, class_total: np.ndarray, alpha: float):
        """Restore `state_arrays()` output; beta is re-derived by the same M-step, so a resumed run is
        bit-identical to an uninterrupted one."""
        if tuple(cw.shape) != tuple(self.cw.shape):
            raise ValueError(f"checkpoint statistics {cw.shape} != engine {tuple(self.cw.shape)}")
        self.cw.copy_(torch.from_numpy(cw).to(self.cw.device, self.cw.dtype))
        # in place: a captured E-step graph holds this buffer's address
        self.class_total.copy_(torch.from_numpy(class_total).to(self.cw.device, torch.float64))
        self._mstep_beta()
        self.alpha = float(alpha)

    def _set_ss_host(self, cw_kv: np.ndarray, normalized=False):
        ct = np.cumsum(cw_kv, axis=1)[:, -1] if cw_kv.shape[1] else np.zeros(self.K)
        if normalized:
            ct = np.ones(self.K)
        cw_t = torch.zeros(self.V, self.KS, dtype=self.cw.dtype)
        cw_t[:, :self.K] = torch.from_numpy(cw_kv.T.copy()).to(self.cw.dtype)
        self.cw.copy_(cw_t.to(self.cw.device))
        ctt = torch.zeros(self.KS, dtype=torch.float64)
        ctt[:self.K] = torch.from_numpy(ct)
        self.class_total.copy_(ctt.to(self.class_total.device))
        self._mstep_beta()

    # ------------------------------------------------------------- E / M steps
    def _mstep_beta(self):
        if self.backend == "hip":
            from ...ops import hip as H
            H.gs_mstep(self.cw, self.class_total, self.beta, self.K)
        else:
            from ...ops import reference as R
            self.beta.copy_(R.mstep(self.cw, self.class_total, self.K))

    def e_step(self):
        """One E-step over the local shard. Returns (lik_sum, alpha_ss_sum) as a device f64 tensor [2]."""
        if self.backend == "hip":
            return self._e_step_hip()
        if self.backend == "torch":
            from ...ops import reference as R
            out = R.estep_jacobi(self.t_doc_ptr, self.t_word, self.t_cnt, self.beta, self.K, self.alpha,
                                 self.var_max_iter, self.settings.var_converged)
            self.gamma = out["gamma"]
            self.iters = out["iters"]
            self.lik = out["lik"]
            if self._chain:
                return self._chain_stats(out)
            if self.emulate_shards > 1:
                return self._emulated_shard_stats(out)
            self.cw = R.suffstats(self.t_doc_ptr, self.t_word, out["e"], out["r"], self.beta, self.V, self.K)
            return torch.stack([out["lik"].sum(), out["alpha_ss"].sum()])
        # cpu: lda-c Gauss-Seidel reference (C++)
        lb = torch.where(self.beta > 0, torch.log(self.beta), torch.full_like(self.beta, LOG_FLOOR))
        res = self._native.lda_estep_ldac(
            self.corpus.doc_ptr, self.corpus.word_idx, self.corpus.counts,
            np.ascontiguousarray(lb.T.numpy()), self.alpha, self.var_max_iter, self.settings.var_converged,
            nshards=self.cpu_shards, threads=_cpu_threads(), gs_updates=resolved_gs_updates(self.settings, self.K))
        self.gamma = torch.from_numpy(res["gamma"])
        self.iters = torch.from_numpy(res["iters"])
        self.lik = torch.from_numpy(res["doc_likelihood"])
        self.cw = torch.from_numpy(np.ascontiguousarray(res["class_word"].T))
        return torch.tensor([res["likelihood"], res["alpha_ss"]], dtype=torch.float64)

    def _chain_stats(self, out):
        """class_word and [likelihood, alpha_ss] as one sequential fold over the corpus in document
        order: this rank continues the fold of the ranks before it (parallel/shardio.chain)."""
        from ...parallel import shardio as SIO
        V, K = self.V, self.K
        lens = (self.t_doc_ptr[1:] - self.t_doc_ptr[:-1]).to(torch.int64)
        doc_of = torch.repeat_interleave(torch.arange(self.D, device=self.device), lens)
        contrib = (out["e"][doc_of][:, :K] * out["r"].unsqueeze(1)).cpu()
        widx = self.t_word.cpu()
        lik = out["lik"].double().cpu().numpy()
        ass = out["alpha_ss"].double().cpu().numpy()

        def fold(carry):
            s = torch.from_numpy(carry[:V * K].reshape(V, K).copy()).index_add_(0, widx, contrib)
            l = np.cumsum(np.concatenate([carry[V * K:V * K + 1], lik]))[-1]
            a = np.cumsum(np.concatenate([carry[V * K + 1:], ass]))[-1]
            return np.concatenate([s.numpy().reshape(-1), [l, a]])

        tot = SIO.chain(self.dist, fold, np.zeros(V * K + 2))
        s = torch.from_numpy(tot[:V * K].reshape(V, K).copy()).to(self.device)
        self.cw = self.beta[:, :K].to(s.dtype) * s
        self._chained = True
        return torch.tensor(tot[V * K:], dtype=torch.float64, device=self.device)

    def _emulated_shard_stats(self, out):
        """class_word and [likelihood, alpha_ss] as N ranks would produce them (each shard's own
        statistics on freshly allocated tensors, then 0 + s_0 + s_1 + ... in shard order)."""
        from ...ops import reference as R
        from ...parallel.dist import engine_bounds
        ptr = self.corpus.doc_ptr
        cw = torch.zeros(self.V, self.K, dtype=torch.float64, device=self.device)
        sc = torch.zeros(2, dtype=torch.float64, device=self.device)
        for d0, d1 in engine_bounds(ptr, self.emulate_shards, self.K):
            e0, e1 = int(ptr[d0]), int(ptr[d1])
            lp = (self.t_doc_ptr[d0:d1 + 1] - self.t_doc_ptr[d0]).clone()
            cw += R.suffstats(lp, self.t_word[e0:e1].clone(), out["e"][d0:d1].clone(), out["r"][e0:e1].clone(),
                              self.beta, self.V, self.K)
            sc += torch.stack([out["lik"][d0:d1].clone().sum(), out["alpha_ss"][d0:d1].clone().sum()])
        self.cw = cw
        return sc

    def _e_step_hip(self):
        """One E-step on the GPU.  The launch sequence (all buckets on their streams, suff-stats,
        reductions) is captured once into a hipGraph and replayed every EM iteration; the
        per-iteration scalars (alpha, lgamma constant, VAR_MAX_ITER) travel in a device buffer."""
        self._push_params()
        if self.use_graph and self._graph is None:
            self._capture_estep()             # its warm-up launch is this call's E-step
        elif self.use_graph:
            self._graph.replay()
        else:
            self._launch_estep()
        self._pushed = None                   # params now hold host values; em_iteration re-checks
        self._ct_fresh = True
        return self._scalars

    def _launch_estep(self, newton_key=None, phase: str = "all"):
        """Enqueue one E-step (``_launch_estep64``): document buckets on their streams, one join, then
        (main stream) the suff-stats launch, which also sums slices of the per-document likelihood /
        alpha_ss, and one column pass giving {likelihood, alpha_ss, class_total}.  With ``newton_key`` =
        (estimate_alpha, num_docs) the M-step follows in the same launch sequence (single-rank fused
        EM iteration): beta, the alpha Newton (workgroup 0) and the EM convergence test in one launch.
        Every kernel is gated on params[DONE] (device-side convergence)."""
        return self._launch_estep64(newton_key, phase)

    def _launch_beta_control(self, newton_key, stages=()):
        """beta, the alpha Newton (workgroup 0 of the same launch) and the EM convergence step [and the
        next E-step's staged rows, trailing workgroups]."""
        from ...ops import hip as H
        rows = self._xchg.local_rows32 if self._xchg is not None else None
        H.gs_mstep_control(self.cw, self.class_total, self.beta, self.K, self._scalars, self._params, self._ctl,
                           self._hist, self._done_count, rows=rows,
                           newton=(newton_key[0], newton_key[1], self._alpha_dummy),
                           stages=stages, word_idx=self.dc.word_idx)

    def _reduce_stats(self):
        """Cross-rank reduction of one EM iteration's statistics (outside the graphs): the packed
        [likelihood, alpha_ss, class_total] doubles by all-reduce, class_word densely by all-reduce
        or sparsely by the all-to-all of shared rows, both in flight together."""
        if self._xchg is None:
            self.dist.allreduce_suffstats(self.cw, self._red)
            return
        import torch.distributed as td
        work = td.all_reduce(self._red, async_op=True)
        self._xchg.exchange()
        work.wait()

    def _launch_mstep(self, estimate_alpha: bool, num_docs: int):
        """M-step on the device after the cross-rank reduction: (sparse exchange: sum the received
        rows), then beta, the alpha Newton and the EM convergence step (one fused launch)."""
        if self._xchg is not None:
            self._xchg.accumulate(self.cw, self._cw_local)
        self._launch_beta_control((estimate_alpha, num_docs))

    def em_iteration(self, estimate_alpha: bool, num_docs: int):
        """One EM iteration (E-step, [all-reduce], M-step, alpha).  Returns (likelihood, alpha_ss)."""
        if self.backend != "hip":
            sc = self.e_step()
            if self._xchg is not None:
                import torch.distributed as td
                red = torch.cat([sc.to(torch.float64), self.cw.sum(0, dtype=torch.float64)])
                tok = self._comm_begin()
                work = td.all_reduce(red, async_op=True)
                local = self._cw_local = self.cw
                self._xchg.pack(local)
                self._xchg.exchange()
                self.cw = torch.zeros_like(local)     # rows of other ranks' words stay 0 (global_rows masks)
                self._xchg.accumulate(self.cw, local)
                work.wait()
                self._comm_end(tok)
                host = red[:2].cpu().tolist()
                self.class_total = red[2:].clone()
                self._mstep_beta()
                if estimate_alpha:
                    self.alpha = special.opt_alpha(float(host[1]), num_docs, self.K)
                return float(host[0]), float(host[1])
            if self.dist is not None and self.dist.active and not self._chain:
                self._cw_local = self.cw.clone()     # this rank's own rows (<rank>.beta)
                tok = self._comm_begin()
                sc = self.dist.allreduce_suffstats(self.cw, sc)
                self._comm_end(tok)
            host = sc.cpu().tolist()
            self.m_step(estimate_alpha, float(host[1]), num_docs)
            return float(host[0]), float(host[1])
        rec = self.em_iterations(1, estimate_alpha, num_docs, stop=False)[0]
        return rec[0], rec[4]

    def em_iterations(self, n: int, estimate_alpha: bool, num_docs: int, likelihood_old: float = 0.0,
                      iteration: int = 0, stop: bool = True, em_converged: Optional[float] = None,
                      em_max_iter: Optional[int] = None) -> List[tuple]:
        """Run up to ``n`` EM iterations with the lda-c convergence test evaluated on the device.

        hip backend: the host enqueues the n iterations (one hipGraph replay each on one rank; E-step
        graph -> RCCL all-reduce -> M-step graph on several) without waiting; after the iteration that
        ends the lda-c loop (``stop``), em_control sets params[DONE] and the kernels of the remaining
        queued iterations return at once.  One read-back per batch returns the executed iterations as
        (likelihood, conv, alpha, var_max_iter, alpha_ss); self.alpha / self.var_max_iter follow the
        last one.  ``likelihood_old`` / ``iteration`` are the loop state before the batch."""
        from ...ops import hip as H
        st = self.settings
        emc = st.em_converged if em_converged is None else em_converged
        emx = st.em_max_iter if em_max_iter is None else em_max_iter
        if self.backend != "hip":
            recs = []
            L_old, i = likelihood_old, iteration
            for _ in range(n):
                lik, ass = self.em_iteration(estimate_alpha, num_docs)
                i += 1
                conv = _conv(L_old, lik)
                if conv < 0:
                    self.var_max_iter = self.var_max_iter * 2
                L_old = lik
                recs.append((lik, conv, self.alpha, self.var_max_iter, ass))
                if stop and not _em_continue(conv, i, emc, emx):
                    break
            return recs
        ticket = self._enqueue_batch(n, estimate_alpha, num_docs, likelihood_old, iteration, stop, emc, emx,
                                     cont=False)
        return self._collect_batch(ticket)

    def em_iterations_pipelined(self, batches: List[int], estimate_alpha: bool, num_docs: int,
                                likelihood_old: float = 0.0, iteration: int = 0, stop: bool = True) -> List[tuple]:
        """``em_iterations`` over several batches with one batch always queued ahead: batch k+1 is
        enqueued before batch k's history is read back, so the GPU never idles on the host's
        read-back, Python bookkeeping and the next batch's launches.  Continuation batches take
        their loop state (previous likelihood, iteration, done flag, alpha, VAR_MAX_ITER) from the
        device, where em_control keeps it; the host sends nothing.  Batches queued after the
        device loop converged are no-ops (every kernel checks params[DONE]).  Not for runs that
        read engine state between batches (LAG saves)."""
        if self.backend != "hip":
            recs = []
            for n in batches:
                r = self.em_iterations(n, estimate_alpha, num_docs, likelihood_old, iteration + len(recs), stop)
                recs += r
                if r:
                    likelihood_old = r[-1][0]
                if len(r) < n:
                    break
            return recs
        st = self.settings
        emc, emx = st.em_converged, st.em_max_iter
        bufs = [self._out_host, torch.zeros_like(self._out_host).pin_memory()]
        recs, pending = [], None
        for j, n in enumerate(batches):
            t = self._enqueue_batch(n, estimate_alpha, num_docs, likelihood_old, iteration, stop, emc, emx,
                                    cont=j > 0, buf=bufs[j % 2])
            if pending is not None:
                r = self._collect_batch(pending)
                recs += r
                if len(r) < pending[2]:       # the device loop ended in that batch: stop enqueuing
                    pending = t
                    break
            pending = t
        if pending is not None:
            recs += self._collect_batch(pending)
        return recs

    def _enqueue_batch(self, n, estimate_alpha, num_docs, likelihood_old, iteration, stop, emc, emx, cont=False,
                       buf=None):
        from ...ops import hip as H
        if n > self._hist_cap:
            raise ValueError(f"batch of {n} EM iterations > history capacity {self._hist_cap}")
        if cont:
            self._ctl[2:3].zero_()   # history slot; loop state and params stay as the device left them
        else:
            if self._pushed != (self.alpha, self.var_max_iter):   # host changed alpha / VAR_MAX_ITER
                self._push_params()
            else:
                self._gate.zero_()
            self._ctl.copy_(torch.tensor([likelihood_old, emc, 0.0, float(iteration), float(emx),
                                          1.0 if stop else 0.0, 0.0, 0.0], dtype=torch.float64))
        key = (bool(estimate_alpha), int(num_docs))
        if not self._distributed:
            self._refill_stages()       # the fused iterations below use staged rows of the current beta
        if not self._distributed and self.use_graph:
            # one rank: one graph per EM iteration (``graph_iters``), cached.  A batch graph (m = the batch)
            # measured the same per iteration (1.82-1.83 ms) but captures a new graph for every new batch
            # size -- inside bench.py's timed window when the warm-up batch differs (2.00 vs 1.82 ms)
            if self._fgraph_key != key:
                self._fgraphs, self._fgraph_key = {}, key
            cap = max(1, int(getattr(self, "graph_iters", 1)))
            left = n
            while left > 0:
                m = min(cap, left)
                g = self._fgraphs.get(m)
                if g is None:
                    # (one more direct launch ahead of the capture, so two iterations are queued while the host
                    # records: measured no faster to convergence, 52.96 vs 53.00 ms median of 7, r6w)
                    self._fgraphs[m] = self._capture(
                        lambda: [self._launch_estep(newton_key=key) for _ in range(m)])
                else:
                    g.replay()
                left -= m
        for _ in range(0 if (not self._distributed and self.use_graph) else n):
            if not self._distributed:
                self._launch_estep(newton_key=key)
            elif self._overlap:
                self._run_phase("A")
                tok = self._comm_begin()
                work = self._xchg.exchange(async_op=True)      # shared rows in flight ...
                self._run_phase("B")                           # ... while the private rows are computed
                import torch.distributed as td
                w2 = td.all_reduce(self._red, async_op=True)
                if work is not None:
                    work.wait()
                w2.wait()
                self._comm_end(tok)
                if not self.use_graph:
                    self._launch_mstep(*key)
                elif self._mgraph_key != key:
                    self._mgraph = self._capture(lambda: self._launch_mstep(*key))
                    self._mgraph_key = key
                else:
                    self._mgraph.replay()
            else:
                if self.use_graph and self._graph is None:
                    self._capture_estep()             # its warm-up launch is this iteration's E-step
                elif self.use_graph:
                    self._graph.replay()
                else:
                    self._launch_estep()
                tok = self._comm_begin()
                self._reduce_stats()
                self._comm_end(tok)
                if not self.use_graph:
                    self._launch_mstep(*key)
                elif self._mgraph_key != key:
                    self._mgraph = self._capture(lambda: self._launch_mstep(*key))
                    self._mgraph_key = key
                else:
                    self._mgraph.replay()
        buf = self._out_host if buf is None else buf
        m = 8 + H.HIST_COLS * n
        buf[:m].copy_(self._ctlhist[:m], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ev, buf, n

    def _collect_batch(self, ticket) -> List[tuple]:
        from ...ops import hip as H
        ev, buf, n = ticket
        t0 = time.perf_counter()
        ev.synchronize()
        self._hphase("wait", t0)
        m = 8 + H.HIST_COLS * n
        out = buf[:m].tolist()
        done = int(out[2])
        rows = [tuple(out[8 + H.HIST_COLS * j: 8 + H.HIST_COLS * j + 5]) for j in range(min(done, n))]
        recs = [(r[0], r[1], r[2], int(r[3]), r[4]) for r in rows]
        if any(r[0] != r[0] for r in recs):
            self._check_split_error()
            bad = next(i for i, r in enumerate(recs) if r[0] != r[0])
            raise RuntimeError(f"EM iteration {bad + 1} of the batch produced a NaN likelihood "
                               f"(schedule: {self.schedule})")
        if recs:
            self.alpha, self.var_max_iter = recs[-1][2], recs[-1][3]
        self._pushed = (self.alpha, self.var_max_iter)
        return recs

    def _push_params(self):
        """Host alpha / VAR_MAX_ITER -> device parameter block.  The lgamma constant is derived
        on the device by the same code the alpha Newton uses, so a run that restarts from host
        values (resume, VAR_MAX_ITER doubling) sees bit-identical parameters."""
        from ...ops import hip as H
        p = torch.zeros(H.PARAM_COUNT, dtype=torch.float64)
        p[0], p[2], p[3] = self.alpha, float(self.var_max_iter), float(self.settings.var_converged)
        self._params.copy_(p)            # pageable source: no pending read of a reused host buffer
        H.alpha_newton(self._scalars, 1.0, self.K, False, self._params, self._alpha_dummy)

    def _check_split_error(self):
        """A NaN likelihood: if a split-document barrier timed out, fail loudly (the kernel
        flags it instead of hanging the GPU)."""
        gp = getattr(self, "gs_plan", None)
        plans = [gp.split if gp is not None else None]
        plans += [w["gp"].split for w in (getattr(self, "_cwin", None) or [])]
        if any(int(b["error"].item()) for x in plans if x is not None for b in x.batches):
            raise RuntimeError("split-document E-step: a cross-workgroup barrier timed out "
                               "(segments of one document were not co-resident)")

    def _capture(self, launch):
        """Run ``launch`` once (this call's real work; first launches also load code objects),
        then capture the same launch sequence into a graph for the following iterations.

        Captured on a dedicated stream with ``capture_begin`` / ``capture_end`` (a private memory pool
        per graph, as ``torch.cuda.graph`` gives) but without its ``gc.collect()`` + ``empty_cache()``
        on entry: those cost ~2 ms per capture and the first EM iteration captures two graphs."""
        launch()
        # the host records the graph while the GPU still runs the real launch (the capture stream waits
        # on the current stream, so replays stay ordered after it): first EM iteration 5.1 -> 3.6 ms
        g = torch.cuda.CUDAGraph()
        if getattr(self, "_capture_stream", None) is None:
            self._capture_stream = torch.cuda.Stream(device=self.device)
        cs = self._capture_stream
        cs.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(cs):
            g.capture_begin()
            try:
                launch()
            finally:
                g.capture_end()
        torch.cuda.current_stream(self.device).wait_stream(cs)
        return g

    def _run_phase(self, phase: str):
        """One of the two E-step graphs of the overlap mode (captured on first use)."""
        attr = "_graph_a" if phase == "A" else "_graph_b"
        g = getattr(self, attr)
        if not self.use_graph:
            self._launch_estep(phase=phase)
        elif g is None:
            setattr(self, attr, self._capture(lambda: self._launch_estep(phase=phase)))
        else:
            g.replay()

    def _capture_estep(self):
        self._graph = self._capture(self._launch_estep)


    def m_step(self, estimate_alpha: bool, alpha_ss: float, num_docs: int):
        """Host M-step of the torch / cpu backends (the hip engine's runs inside its launch sequence)."""
        self.class_total = self.cw.sum(0, dtype=torch.float64)
        self._mstep_beta()
        if estimate_alpha:
            self.alpha = special.opt_alpha(alpha_ss, num_docs, self.K)

    # -------------------------------------------------------------- outputs
    def log_beta(self, cw: Optional[torch.Tensor] = None) -> np.ndarray:
        """[K, V] float64 log p(w|z) as lda-c would save it (-100 floor).  Collective under the
        sparse exchange unless ``cw`` (a ``global_cw()`` result) is given."""
        cw = (self.global_cw() if cw is None else cw)[:, :self.K]
        return _log_beta_host(cw, self.class_total[:self.K])

    # outputs up to this size are copied behind the device work (pinned buffer + event) by the
    # *_deferred variants; larger ones take the blocking, chunked path
    DEFER_BYTES = 256 << 20

    def log_beta_deferred(self, cw: Optional[torch.Tensor] = None, reuse: bool = False):
        """(host [K, V] array, event or None): ``log_beta`` whose device-to-host copy is queued on the
        current stream into a pinned buffer; the array is valid once ``event`` completed.  The LAG saves
        hand both to the file writer, so an EM run with saves does not wait for each copy.  ``reuse``: the
        buffer comes from the process's PinnedPool (the caller must not keep the array past its writer
        jobs' use -- the LAG saves; the final save's arrays are returned to the caller and stay fresh)."""
        full = self.global_cw() if cw is None else cw
        c = full[:, :self.K]
        V, K = c.shape
        if self.device.type != "cuda" or K * V * 8 > self.DEFER_BYTES:
            return _log_beta_host(c, self.class_total[:K]), None
        lb = self._log_beta_device(full, K)
        host, arr = _pinned(reuse, (K, V), torch.float64)
        host.copy_(lb, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return arr, ev

    def _log_beta_device(self, full: torch.Tensor, K: int) -> torch.Tensor:
        """[K, V] saved log beta on the device: the HIP kernel (ops/hip.py log_beta_t) where the engine is the HIP
        one and the statistics are plain contiguous fp64, else torch's transpose / log / where (the same bits)."""
        ct = self.class_total
        if self.backend == "hip" and full.dtype == torch.float64 and full.is_contiguous() and \
                ct.dtype == torch.float64 and ct.is_contiguous():
            from ...ops import hip as H
            return H.log_beta_t(full, ct, K, LOG_FLOOR)
        cT = full[:, :K].T.to(torch.float64).contiguous()
        lct = torch.log(ct[:K].to(torch.float64))
        return torch.where(cT > 0, torch.log(cT) - lct[:, None], torch.full_like(cT, LOG_FLOOR))

    def save_handoff(self, cw: torch.Tensor, gamma: bool, checkpoint: bool) -> Optional[dict]:
        """A LAG save's state as DeviceHandoffs -- log_beta [K, V], gamma [D, K] (``gamma``), the checkpoint's
        class_word and class totals (``checkpoint``) -- copied on the device behind the work already queued, one
        event for all; None where the handoff does not apply (not the one-rank HIP engine on a GPU, or a save
        larger than SNAPSHOT_BYTES: those keep the pinned-copy path)."""
        if self.backend != "hip" or self.device.type != "cuda" or self._distributed:
            return None
        K = self.K
        nbytes = (K * cw.shape[0] + (self.gamma.shape[0] * K if gamma else 0) +
                  (cw.numel() + self.class_total.numel() if checkpoint else 0)) * 8
        if nbytes > self.SNAPSHOT_BYTES:
            return None
        out = dict(log_beta=self._log_beta_device(cw, K))
        if gamma:
            out["gamma"] = self.gamma[:, :K].contiguous() if self.gamma.shape[1] != K else self.gamma.clone()
        if checkpoint:
            out["cw"] = cw.clone()
            out["class_total"] = self.class_total.clone()
        ev = torch.cuda.Event()
        ev.record()
        return {k: DeviceHandoff(v, ev) for k, v in out.items()}

    def host_copy_deferred(self, t: torch.Tensor, reuse: bool = False):
        """(host array, event or None): a copy of device tensor ``t`` queued on the current stream into a
        pinned buffer (valid once ``event`` completed); blocking for host tensors or above DEFER_BYTES."""
        if t.device.type != "cuda" or t.numel() * t.element_size() > self.DEFER_BYTES:
            return t.to("cpu", copy=True).numpy(), None
        host, arr = _pinned(reuse, tuple(t.shape), t.dtype)
        host.copy_(t if t.is_contiguous() else t.contiguous(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return arr, ev

    def local_gamma_deferred(self, reuse: bool = False):
        """(host [D_local, K] gamma, event or None): ``local_gamma`` with a queued pinned copy."""
        g = self.gamma[:, :self.K]
        if self.device.type != "cuda" or g.numel() * 8 > self.DEFER_BYTES:
            return self.local_gamma(), None
        host, arr = _pinned(reuse, tuple(g.shape), torch.float64)
        host.copy_(g if g.is_contiguous() else g.contiguous(), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return arr, ev

    def local_log_beta(self) -> np.ndarray:
        """[K, V] log of this rank's own class_word rows over the GLOBAL class totals (-100 floor):
        the per-worker ``<rank>.beta`` (README.md:121), final.beta = log(sum over ranks of exp)."""
        local = getattr(self, "_cw_local", None)
        cw = (self.cw if local is None else local)[:, :self.K]
        return _log_beta_host(cw, self.class_total[:self.K].to(cw.device))

    def word_assignments(self) -> np.ndarray:
        """run_em's final pass: a fresh E-step of every document under the current
        (final) model, then for every corpus entry of this rank the topic of its largest phi, the first
        maximum (lda-c write_word_assignment).  Overwrites gamma and the per-document state: read the
        model and gamma first.  Returns int64 [nnz] in corpus entry order.

        fp64 HIP engine: the document kernels alone (no sufficient statistics), whose final pass leaves
        c_n phi_nk = E_jk b_nk c_n / P_n -- phi of each word under its chunk's gamma, as lda-c's
        sequential pass leaves phi[n] -- in the c.phi rows; torch backend: Jacobi phi = E_k b_kn / P_n;
        cpu backend: psi(gamma) + log beta with the fresh gamma."""
        K = self.K
        if self.backend == "hip" and self.fp64:
            self._push_params()
            z = torch.empty(self.corpus.nnz, dtype=torch.int64, device=self.device)
            step = 1 << 22
            wins = self._cwin or [dict(gp=None, e0=0, e1=self.corpus.nnz)]
            for w in wins:
                if w["gp"] is None:
                    self._launch_estep64(phase="estep")
                else:
                    self._launch_buckets(w["gp"], win=w)
                for a in range(w["e0"], w["e1"], step):
                    b = min(w["e1"], a + step)
                    z[a:b] = torch.argmax(self.cphi[a - w["e0"]:b - w["e0"], :K], dim=1)
            return z.cpu().numpy()
        if self.backend == "torch":
            from ...ops import reference as R
            out = R.estep_jacobi(self.t_doc_ptr, self.t_word, self.t_cnt, self.beta, K, self.alpha,
                                 self.var_max_iter, self.settings.var_converged)
            lens = (self.t_doc_ptr[1:] - self.t_doc_ptr[:-1]).to(torch.int64)
            doc_of = torch.repeat_interleave(torch.arange(self.D, device=self.device), lens)
            return torch.argmax(out["e"][doc_of][:, :K] * self.beta[self.t_word, :K], dim=1).cpu().numpy()
        if self.backend == "cpu":
            lb = torch.where(self.beta > 0, torch.log(self.beta), torch.full_like(self.beta, LOG_FLOOR))
            return self._native.lda_assign_ldac(self.corpus.doc_ptr, self.corpus.word_idx,
                                                self.corpus.counts.astype(np.float64), np.ascontiguousarray(lb.T.numpy()),
                                                self.alpha, self.var_max_iter, self.settings.var_converged,
                                                gs_updates=resolved_gs_updates(self.settings, self.K)).astype(np.int64)
        raise NotImplementedError(f"word assignments for backend {self.backend} / {self.precision}")

    def local_gamma(self) -> np.ndarray:
        g = self.gamma[:, :self.K]
        # padded topics (KS > K): made contiguous on the device, so the D2H copy is one block
        return (g if g.is_contiguous() else g.contiguous()).to("cpu", torch.float64, copy=True).numpy()

    def gather_gamma(self) -> np.ndarray:
        g = self.local_gamma()
        if self.dist is not None and self.dist.active:
            return self.dist.gather_rows(g, self.global_docs)
        return g

    def _hphase(self, name: str, t0: float):
        """Host seconds of one EM-loop phase since ``t0`` (init / enqueue / wait / save / save_final), summed
        per run into ``host_phases``: where the thread driving the GPU spends the lda stage."""
        hp = self.__dict__.setdefault("host_phases", {})
        hp[name] = hp.get(name, 0.0) + time.perf_counter() - t0

    # ----------------------------------------------------- LAG saves, pipelined
    SNAPSHOT_BYTES = 1 << 30     # device snapshots of the LAG state (2 sets) only below this size

    def _snapshot_saves_ok(self) -> bool:
        """One rank, fp64 HIP engine, graphs: LAG saves from device snapshots (2 x (cw + gamma) bytes)."""
        if self.backend != "hip" or self._distributed or not self.use_graph or self._cwin is not None:
            return False
        return 2 * (self.cw.numel() + self.gamma.numel()) * 8 <= self.SNAPSHOT_BYTES

    def _em_with_snapshots(self, on_save, on_iteration, i, L_old, hist, stats, lag, n_docs_global):
        """EM iterations with LAG saves and one batch queued ahead: a batch ending on a LAG boundary is
        followed on the stream by copies of class_word, the class totals and gamma into one of two
        snapshot sets; once its history is read back (the next batch already queued) the save runs from
        the snapshot, with the host scalars of that iteration.  A batch the device loop stopped early (the
        loop converged before the boundary) saves nothing, exactly as the draining loop would not."""
        st = self.settings
        # lda-c's loop test runs after each iteration while i <= EM_MAX_ITER: up to EM_MAX_ITER + 1 iterations
        batches = _lag_batches(i, st.em_max_iter + 1, lag, self.max_batch)
        if not batches:
            return i, L_old, 1.0
        if getattr(self, "_snaps", None) is None:
            self._snaps = [tuple(torch.empty_like(x) for x in (self.cw, self.class_total, self.gamma))
                           for _ in range(2)]
        emc, emx = st.em_converged, st.em_max_iter
        bufs = [self._out_host, torch.zeros_like(self._out_host).pin_memory()]
        conv = 1.0
        pending = None          # (ticket, batch size, snapshot set or None)
        it_q = i

        def collect(p):
            nonlocal i, L_old, conv
            ticket, n, snap = p
            recs = self._collect_batch(ticket)
            for lik, c, alpha, vmi, _ass in recs:
                i += 1
                L_old, conv = lik, c
                hist.append((lik, c))
                stats.append(EMIterStats(i, lik, c, alpha, 0.0, -1.0, -1, vmi))
                if on_iteration is not None:
                    on_iteration(self, i, lik, c)
            if snap is not None and len(recs) == n and i % lag == 0:
                view = _Snapshot(self, *snap)
                t0 = time.perf_counter()
                on_save(f"{i:03d}", view)
                self._hphase("save", t0)
            return len(recs) < n

        for j, n in enumerate(batches):
            t0 = time.perf_counter()
            t = self._enqueue_batch(n, st.estimate_alpha, n_docs_global, L_old, it_q, True, emc, emx,
                                    cont=j > 0, buf=bufs[j % 2])
            self._hphase("enqueue", t0)
            it_q += n
            snap = None
            if it_q % lag == 0:
                snap = self._snaps[j % 2]
                for dst, src in zip(snap, (self.cw, self.class_total, self.gamma)):
                    dst.copy_(src, non_blocking=True)
            if pending is not None:
                if collect(pending):     # the device loop ended in that batch: this one is a no-op
                    pending = (t, n, snap)
                    break
            pending = (t, n, snap)
        if pending is not None:
            collect(pending)
        return i, L_old, conv

    # ----------------------------------------------------------------- driver
    def run(self, start: str = "random", corpus_global: Optional[Corpus] = None,
            on_iteration: Optional[Callable] = None, on_save: Optional[Callable] = None,
            start_iteration: int = 0, likelihood_old: float = 0.0, verbose: bool = False) -> LDAResult:
        """Run EM to convergence. `on_save(tag, engine)` fires for '000', every LAG and 'final'."""
        st = self.settings
        lag = st.lag
        t0 = time.perf_counter()
        self.host_phases = {}
        if start == "random":
            self.init_random()
        elif start == "seeded":
            self.init_seeded(corpus_global)
        elif start == "resume":
            pass  # state restored by caller (checkpoint.restore)
        else:
            raise ValueError(start)
        self._hphase("init", t0)
        if on_save is not None and start_iteration == 0:
            ts = time.perf_counter()
            on_save("000", self)
            self._hphase("save", ts)
        i = start_iteration
        L_old = likelihood_old
        conv = 1.0
        hist = []
        stats = []
        n_docs_global = self.global_docs
        per_iter_stats = verbose or self.collect_iter_stats   # an extra D2H copy per iteration: opt-in
        if on_save is None and not per_iter_stats and self.backend == "hip" and \
                _em_continue(conv, i, st.em_converged, st.em_max_iter):
            # no saves: batches run back to back with one queued ahead (em_iterations_pipelined)
            left = st.em_max_iter - i + 1
            batches = [min(self.pipe_batch, left - b) for b in range(0, max(left, 0), self.pipe_batch)]
            ti = time.perf_counter()
            recs = self.em_iterations_pipelined(batches, st.estimate_alpha, n_docs_global, likelihood_old=L_old,
                                                iteration=i)
            dt = (time.perf_counter() - ti) / max(len(recs), 1)
            for lik, conv, alpha, vmi, _ass in recs:
                i += 1
                L_old = lik
                hist.append((lik, conv))
                stats.append(EMIterStats(i, lik, conv, alpha, dt, -1.0, -1, vmi))
                if on_iteration is not None:
                    on_iteration(self, i, lik, conv)
            conv = 0.0 if not recs else conv
        if on_save is not None and lag > 0 and not per_iter_stats and self._snapshot_saves_ok() and \
                _em_continue(conv, i, st.em_converged, st.em_max_iter):
            # LAG saves without draining the device: batches end on LAG boundaries, each followed by an
            # on-device snapshot of the saved state, one batch always queued ahead (_em_with_snapshots)
            i, L_old, conv = self._em_with_snapshots(on_save, on_iteration, i, L_old, hist, stats, lag,
                                                     n_docs_global)
        while on_save is not None or per_iter_stats or self.backend != "hip":
            if not _em_continue(conv, i, st.em_converged, st.em_max_iter):
                break
            # One batch = the iterations up to the next LAG save (the saved state must be that
            # iteration's), at most max_batch; the device stops the batch itself on convergence.
            n = 1 if per_iter_stats else self.max_batch
            if on_save is not None and lag > 0:
                n = min(n, lag - (i % lag))
            n = max(1, min(n, st.em_max_iter - i + 1))
            ti = time.perf_counter()
            range_push(f"em_iters_{i + 1}_{i + n}")
            recs = self.em_iterations(n, st.estimate_alpha, n_docs_global, likelihood_old=L_old, iteration=i)
            range_pop()
            dt = (time.perf_counter() - ti) / max(len(recs), 1)
            if per_iter_stats:
                it_np = self.iters.cpu().numpy() if isinstance(self.iters, torch.Tensor) else np.asarray(self.iters)
                it_mean = float(it_np.mean()) if it_np.size else 0.0
                it_max = int(it_np.max()) if it_np.size else 0
            else:
                it_mean, it_max = -1.0, -1
            for lik, conv, alpha, vmi, _ass in recs:
                i += 1
                L_old = lik
                hist.append((lik, conv))
                stt = EMIterStats(i, lik, conv, alpha, dt, it_mean, it_max, vmi)
                stats.append(stt)
                if verbose:
                    print(f"**** em iteration {i} **** L={lik:.6f} conv={conv:.5e} alpha={alpha:.5f} "
                          f"var_iters(mean/max)={stt.var_iter_mean:.2f}/{stt.var_iter_max} {dt*1e3:.2f} ms",
                          flush=True)
                if on_iteration is not None:
                    on_iteration(self, i, lik, conv)
            if not recs:
                break
            if on_save is not None and lag > 0 and (i % lag) == 0:
                on_save(f"{i:03d}", self)
        if on_save is not None:
            ts = time.perf_counter()
            on_save("final", self)
            self._hphase("save_final", ts)
        res = LDAResult(log_beta=None, gamma=None, alpha=self.alpha, num_topics=self.K, num_terms=self.V,
                        likelihoods=hist, stats=stats, em_iterations=i, seconds=time.perf_counter() - t0)
        return res


class _Snapshot:
    """The saved state of one LAG iteration, copied on the device behind that iteration's batch (class_word,
    class totals, gamma) plus its host scalars; duck-types the engine for estimate()'s on_save (the state
    methods read the snapshot, everything else falls through to the engine)."""

    def __init__(self, eng, cw, class_total, gamma):
        self._eng, self.cw, self._cw_local, self.class_total, self.gamma = eng, cw, cw, class_total, gamma
        self.alpha, self.var_max_iter = eng.alpha, eng.var_max_iter

    def __getattr__(self, name):
        return getattr(self._eng, name)

    def global_cw(self):
        return self.cw

    log_beta_deferred = LDAEngine.log_beta_deferred
    _log_beta_device = LDAEngine._log_beta_device
    save_handoff = LDAEngine.save_handoff
    host_copy_deferred = LDAEngine.host_copy_deferred
    local_gamma_deferred = LDAEngine.local_gamma_deferred
    local_gamma = LDAEngine.local_gamma


def _pinned(reuse: bool, shape, dtype):
    """(pinned tensor, its ndarray): from the PinnedPool when ``reuse``, else a fresh buffer."""
    if reuse:
        return _PINNED.take(shape, dtype)
    t = torch.empty(shape, dtype=dtype, pin_memory=True)
    return t, t.numpy()


def _lag_batches(i: int, last: int, lag: int, cap: int) -> List[int]:
    """Batch sizes covering iterations i + 1 .. last, each ending at a multiple of ``lag`` or the end,
    at most ``cap`` long."""
    out = []
    while i < last:
        n = min(cap, lag - (i % lag), last - i)
        out.append(n)
        i += n
    return out


def resolved_gs_updates(settings, K: int) -> int:
    """settings.gs_updates with -1 (the parity mode) resolved for K; 0 stays 0 (the CPU engine's
    literal per-word schedule, the GPU engine's default 32)."""
    u = int(settings.gs_updates)
    return parity_gs_updates(K) if u < 0 else u


def parity_gs_updates(K: int) -> int:
    """The U per K that meets lda-c parity on the BASELINE configs (profiles/r3_precision_parity.md:
    >= 85 % overlap of the 0.1 % most suspicious entries, alpha <= 1 %, final likelihood <= 1e-4;
    K = 100 reaches 82-84 % overlap from U = 1024 on, with alpha and the likelihood within 1e-5)."""
    if K <= 32:
        return 32
    if K <= 52:
        return 64          # K = 50: 94.5 % overlap; the split kernel keeps 64-row tables (5.6 ms / EM iteration)
    return 1024


def _log_beta_host(cw: torch.Tensor, ct: torch.Tensor, elems: int = 1 << 25) -> np.ndarray:
    """[K, V] float64 host array of log(cw) - log(ct) (-100 floor where cw == 0), computed in blocks of
    topics: each block is transposed on the device into [k, V] rows, so it lands in its contiguous rows
    of the host array with one copy (a block of words lands in K strided pieces), and the device
    transient stays ~``elems`` doubles instead of V x K temporaries (3.6 GB each at config 5)."""
    V, K = cw.shape
    out = np.empty((K, V), np.float64)
    if V == 0 or K == 0:
        return out
    lct = torch.log(ct.to(torch.float64))
    host = torch.from_numpy(out)
    kb = max(1, min(K, elems // max(V, 1)))
    for k0 in range(0, K, kb):
        k1 = min(K, k0 + kb)
        c = cw[:, k0:k1].T.to(torch.float64).contiguous()          # [k, V], transposed on the device
        lb = torch.where(c > 0, torch.log(c) - lct[k0:k1, None], torch.full_like(c, LOG_FLOOR))
        host[k0:k1].copy_(lb)                                       # one contiguous D2H copy
    return out


def _conv(L_old: float, lik: float) -> float:
    """lda-c: converged = (likelihood_old - likelihood) / likelihood_old (IEEE semantics at 0)."""
    if L_old != 0:
        return (L_old - lik) / L_old
    return math.inf if lik < 0 else (-math.inf if lik > 0 else math.nan)


def _em_continue(conv: float, i: int, em_converged: float, em_max_iter: int) -> bool:
    """lda-c run_em loop condition after iteration i."""
    return ((conv < 0) or (conv > em_converged) or (i <= 2)) and (i <= em_max_iter)
