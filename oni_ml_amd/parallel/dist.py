"""Process-group context: one process per GPU, RCCL over xGMI (torch backend "nccl").

Replaces the reference's MPI layer (`mpiexec -n 20 -f machinefile ./lda est ...`,
ml_ops.sh:80):

* documents are sharded CONTIGUOUSLY and balanced by nnz (not doc count), so the
  per-rank gamma blocks concatenate in corpus order exactly like lda-c's
  per-worker <rank>.gamma files combined into final.gamma (README.md:121);
* per EM iteration the collectives are the class_word reduction and one small
  f64 all-reduce ([likelihood, alpha ss, class_total]).  class_word is reduced
  either densely (ring all-reduce of [V x KS] f64, K*V*8 bytes) or -- when the
  ranks' vocabularies overlap little, as IP/port "words" of different days do --
  by `VocabExchange`: an all-to-all of only the rows two ranks share.  On the
  fully connected xGMI mesh an all-to-all uses every link at once, while a ring
  all-reduce is bound by one link per step;
* the CPU test path runs the same code over gloo.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import knobs

# ordered_allreduce's slice per rank (MiB): N x the slice of extra memory, not N full copies
ORDERED_CHUNK_MB = 256


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    # ONI_DIST_DETERMINISTIC=1: sufficient statistics are reduced by all-gather + a sum in rank order
    # (0 + s_0 + s_1 + ...), the order a single process emulating the same shards uses
    # (LDAEngine(emulate_shards=N)), so an N-rank run is bitwise equal to that single-process run.
    # The default ring all-reduce is bitwise identical on every rank but its association differs.
    deterministic: bool = False
    # ONI_DIST_FORCE_GROUP=1: a process group even for one rank -- every distributed code path (the
    # collectives, the sharded pipeline) then runs, e.g. one-rank RCCL on a one-GPU box
    forced: bool = False

    @property
    def initialized(self) -> bool:
        return (self.world_size > 1 or self.forced) and torch.distributed.is_initialized()

    @property
    def active(self) -> bool:
        """The multi-rank code paths apply: several ranks, or a forced one-rank group."""
        return self.world_size > 1 or self.forced

    # -------------------------------------------------------------- sharding
    def shard_range(self, corpus, K: int = None):
        """This rank's documents of a corpus every rank holds whole (strong scaling): ``engine_bounds``,
        the one shard rule every consumer of a rank's document range uses."""
        return engine_bounds(corpus.doc_ptr, self.world_size, K)[self.rank]

    # ----------------------------------------------------------- collectives
    def allreduce_suffstats(self, cw: torch.Tensor, scalars: torch.Tensor) -> torch.Tensor:
        if not self.initialized:
            return scalars
        import torch.distributed as td

        if self.deterministic:
            self.ordered_allreduce(scalars)
            self.ordered_allreduce(cw)
            return scalars
        work = td.all_reduce(scalars, async_op=True)
        td.all_reduce(cw)
        work.wait()
        return scalars

    def ordered_allreduce(self, t: torch.Tensor) -> torch.Tensor:
        """In place: t <- 0 + t_0 + t_1 + ... + t_{N-1} (rank order) on every rank.

        Gathered in slices of <= ORDERED_CHUNK_MB (256) MiB per rank, so the extra memory is
        N x the slice, not N full copies (a config-5 class_word is 3.8 GB per copy)."""
        import torch.distributed as td

        flat = t.view(-1) if t.is_contiguous() else t.contiguous().view(-1)
        step = max(1, int(ORDERED_CHUNK_MB * 2**20) // max(1, t.element_size()))
        step = min(step, max(1, flat.numel()))
        parts = [torch.empty(step, dtype=t.dtype, device=t.device) for _ in range(self.world_size)]
        for a in range(0, flat.numel(), step):
            b = min(flat.numel(), a + step)
            views = [p[:b - a] for p in parts]
            td.all_gather(views, flat[a:b].contiguous())
            acc = torch.zeros(b - a, dtype=t.dtype, device=t.device)
            for v in views:
                acc += v
            flat[a:b] = acc
        if flat.data_ptr() != t.data_ptr():
            t.copy_(flat.view_as(t))
        return t

    def self_check(self):
        """Start-up check of the collective path (RCCL on GPUs): an all-reduce, a device-scoped barrier
        and an all_to_all_single with known answers.  Raises with the backend and device named, instead
        of letting the first EM iteration hang or return garbage."""
        if not self.initialized:
            return
        import torch.distributed as td

        dev = self._coll_device()
        N, r = self.world_size, self.rank
        try:
            x = torch.full((4,), float(r + 1), dtype=torch.float64, device=dev)
            td.all_reduce(x)
            want = N * (N + 1) / 2
            if not bool((x == want).all()):
                raise RuntimeError(f"all_reduce returned {x.tolist()}, expected {want}")
            self.barrier()
            send = torch.arange(N, dtype=torch.float64, device=dev) + 100.0 * r
            recv = torch.empty_like(send)
            td.all_to_all_single(recv, send)
            exp = torch.arange(N, dtype=torch.float64, device=dev) * 100.0 + r
            if not torch.equal(recv, exp):
                raise RuntimeError(f"all_to_all_single returned {recv.tolist()}, expected {exp.tolist()}")
        except Exception as e:
            raise RuntimeError(f"collective self-check failed on rank {r}/{N} (backend {self.backend}, "
                               f"device {dev}): {e}") from e

    def allreduce_int(self, v: int) -> int:
        if not self.initialized:
            return int(v)
        import torch.distributed as td

        t = torch.tensor([int(v)], dtype=torch.int64, device=self._coll_device())
        td.all_reduce(t)
        return int(t.item())

    def allreduce_max(self, v: float) -> float:
        if not self.initialized:
            return float(v)
        import torch.distributed as td

        t = torch.tensor([float(v)], dtype=torch.float64, device=self._coll_device())
        td.all_reduce(t, op=td.ReduceOp.MAX)
        return float(t.item())

    def broadcast_object(self, obj):
        if not self.initialized:
            return obj
        import torch.distributed as td

        lst = [obj]
        td.broadcast_object_list(lst, src=0)
        return lst[0]

    def gather_rows(self, local: np.ndarray, total_rows: int) -> np.ndarray:
        """All-gather contiguous row blocks in rank order (order-preserving combine)."""
        if not self.initialized:
            return local
        import torch.distributed as td

        dev = self._coll_device()
        n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(n) for _ in range(self.world_size)]
        td.all_gather(sizes, n)
        sizes = [int(s.item()) for s in sizes]
        mx = max(sizes)
        buf = torch.zeros((mx,) + local.shape[1:], dtype=torch.float64, device=dev)
        buf[: local.shape[0]] = torch.from_numpy(np.ascontiguousarray(local, dtype=np.float64)).to(dev)
        outs = [torch.zeros_like(buf) for _ in range(self.world_size)]
        td.all_gather(outs, buf)
        res = np.concatenate([o[:s].cpu().numpy() for o, s in zip(outs, sizes)], axis=0)
        assert res.shape[0] == total_rows, (res.shape, total_rows)
        return res

    def broadcast_corpus(self, corpus):
        """Rank 0's Corpus on every rank (arrays via the collective backend, not pickles)."""
        if not self.initialized:
            return corpus
        import torch.distributed as td
        from ..corpus.csr import Corpus

        meta = [None]
        if self.rank == 0:
            meta = [(corpus.num_docs, corpus.nnz, corpus.num_terms)]
        td.broadcast_object_list(meta, src=0)
        D, nnz, V = meta[0]
        dev = self._coll_device()
        if self.rank == 0:
            ptr = torch.from_numpy(corpus.doc_ptr).to(dev)
            w = torch.from_numpy(corpus.word_idx).to(dev)
            c = torch.from_numpy(corpus.counts).to(dev)
        else:
            ptr = torch.empty(D + 1, dtype=torch.int64, device=dev)
            w = torch.empty(nnz, dtype=torch.int32, device=dev)
            c = torch.empty(nnz, dtype=torch.int64, device=dev)
        for t in (ptr, w, c):
            td.broadcast(t, src=0)
        if self.rank == 0:
            return corpus
        return Corpus(ptr.cpu().numpy(), w.cpu().numpy(), c.cpu().numpy(), V)

    def barrier(self):
        if self.initialized:
            import torch.distributed as td

            if self.backend == "nccl":
                td.barrier(device_ids=[self.local_rank])
            else:
                td.barrier()

    def shutdown(self):
        if self.initialized:
            import torch.distributed as td

            td.destroy_process_group()

    def _coll_device(self):
        return self.device if self.backend == "nccl" else torch.device("cpu")


class VocabExchange:
    """Sparse cross-rank reduction of class_word rows.

    A rank's E-step only produces class_word rows for words of its own documents,
    and its next E-step only reads beta rows of those words; beta[w] needs the
    global sum of row w over the ranks that hold w.  With L_r the sorted word list
    of rank r, the plan (built once) is the intersections L_r ∩ L_s; every EM
    iteration each rank

      1. packs its rows of L_r ∩ L_s for every s (``pack``, graph-capturable),
      2. exchanges them with one ``all_to_all_single`` (``exchange``),
      3. sums, for its own words, the contributions in global rank order
         (``accumulate``: 0 + c_0 + c_1 + ... -- every rank that holds w
         therefore gets bitwise the same sum, like an all-reduce).

    Rows of words a rank does not hold are left zero; ``global_rows`` (dense,
    masked by a single owner per word) rebuilds the full matrix for model files.
    Traffic per rank: sum_s |L_r ∩ L_s| rows instead of 2 (N-1)/N V rows."""

    def __init__(self, ctx: "DistContext", local_words: np.ndarray, V: int, width: int, device, dtype):
        import torch.distributed as td

        self.ctx, self.V, self.width = ctx, int(V), int(width)
        self.device, self.dtype = torch.device(device), dtype
        cdev = ctx._coll_device()
        lw = torch.as_tensor(np.asarray(local_words, dtype=np.int64), device=cdev)
        n = torch.tensor([lw.numel()], dtype=torch.int64, device=cdev)
        sizes = [torch.zeros_like(n) for _ in range(ctx.world_size)]
        td.all_gather(sizes, n)
        sizes = [int(x.item()) for x in sizes]
        pad = torch.full((max(sizes),), -1, dtype=torch.int64, device=cdev)
        pad[: lw.numel()] = lw
        lists = [torch.empty_like(pad) for _ in range(ctx.world_size)]
        td.all_gather(lists, pad)
        lists = [l[:k].cpu() for l, k in zip(lists, sizes)]
        mine = lists[ctx.rank]
        self.common = []
        for s_, other in enumerate(lists):
            if s_ == ctx.rank:
                self.common.append(torch.zeros(0, dtype=torch.int64))
            else:
                self.common.append(mine[torch.isin(mine, other)])
        self.splits = [int(c.numel()) for c in self.common]
        self.rows = sum(self.splits)
        # single owner per word (lowest rank holding it): the dense model-file reduction
        owner = torch.full((self.V,), ctx.world_size, dtype=torch.int64)
        for s_ in reversed(range(ctx.world_size)):
            owner[lists[s_]] = s_
        self.owned = (owner == ctx.rank).to(self.device)
        self.send_idx = torch.cat(self.common).to(self.device)
        self.recv_idx = [c.to(self.device) for c in self.common]
        # this rank's own words: the rows accumulate() writes and the M-step needs
        self.local_ids = mine.to(self.device)
        self.local_rows32 = self.local_ids.to(torch.int32)
        self.offsets = np.concatenate([[0], np.cumsum(self.splits)]).tolist()
        # accumulate() plan, CSR over this rank's words: each row's sources in rank order
        # (src >= 0: a received row, -1: the rank's own row)
        n_loc = int(mine.numel())
        if n_loc > 1 and not bool((mine[1:] > mine[:-1]).all()):
            raise ValueError("VocabExchange: local word list must be sorted and unique")
        r_rows, r_key, r_src = [], [], []
        for s_ in range(ctx.world_size):
            if s_ == ctx.rank:
                rr = torch.arange(n_loc, dtype=torch.int64)
                ss = torch.full((n_loc,), -1, dtype=torch.int64)
            else:
                rr = torch.searchsorted(mine, self.common[s_])
                ss = int(self.offsets[s_]) + torch.arange(self.splits[s_], dtype=torch.int64)
            r_rows.append(rr)
            r_key.append(rr * ctx.world_size + s_)
            r_src.append(ss)
        key = torch.cat(r_key)
        order = torch.argsort(key, stable=True)
        rows_sorted = torch.cat(r_rows)[order]
        src = torch.cat(r_src)[order]
        ptr = torch.zeros(n_loc + 1, dtype=torch.int64)
        ptr[1:] = torch.cumsum(torch.bincount(rows_sorted, minlength=n_loc), 0)
        if src.numel() and int(src.max()) >= max(self.rows, 1):
            raise RuntimeError("VocabExchange: accumulate plan out of range")
        self.acc_ptr = ptr.to(torch.int32).to(self.device)
        self.acc_src = src.to(torch.int32).to(self.device)
        self.send = torch.zeros(max(self.rows, 1), self.width, dtype=dtype, device=self.device)
        self.recv = torch.zeros_like(self.send)
        self.local_words = int(mine.numel())
        mx = torch.tensor([self.rows], dtype=torch.int64, device=cdev)
        td.all_reduce(mx, op=td.ReduceOp.MAX)
        self.max_rows = int(mx.item())

    def worthwhile(self) -> bool:
        """The busiest rank's all-to-all rows (sent = received) against a ring all-reduce's
        2 (N-1)/N V rows per rank, with a margin for the all-to-all's per-peer latency.
        Identical on every rank (max over ranks)."""
        N = self.ctx.world_size
        return self.max_rows < 0.7 * 2.0 * (N - 1) / N * self.V

    def pack(self, cw_local: torch.Tensor):
        if self.rows:
            torch.index_select(cw_local, 0, self.send_idx, out=self.send[: self.rows])

    def exchange(self, async_op: bool = False):
        """Collective: every rank calls it every EM iteration (possibly with no rows)."""
        import torch.distributed as td

        if self.ctx.backend != "nccl" and self.send.device.type == "cuda":
            # gloo rehearsal of several ranks on one GPU: stage through host memory
            s_cpu = self.send[: self.rows].cpu()
            r_cpu = torch.empty_like(s_cpu)
            td.all_to_all_single(r_cpu, s_cpu, self.splits, self.splits)
            self.recv[: self.rows].copy_(r_cpu)
            return None
        return td.all_to_all_single(self.recv[: self.rows], self.send[: self.rows], self.splits, self.splits,
                                    async_op=async_op)

    def accumulate(self, cw_out: torch.Tensor, cw_local: torch.Tensor):
        """cw_out[w] = 0 + c_0[w] + c_1[w] + ... for this rank's words w (rank order); rows of other
        words are not touched (never read on this rank).  Cost ~ local rows, not the union vocabulary."""
        if cw_out.is_cuda and cw_out.dtype == torch.float64 and self.width % 2 == 0:
            # one HIP launch (csrc/hip/reduce.hip rows_accumulate_kernel), the same bits as the loop below
            from ..ops import hip as H
            H.rows_accumulate(self.local_rows32, self.acc_ptr, self.acc_src, cw_local, self.recv, cw_out)
            return
        li = self.local_ids
        cw_out.index_fill_(0, li, 0)
        for s_ in range(self.ctx.world_size):
            if s_ == self.ctx.rank:
                cw_out.index_add_(0, li, cw_local.index_select(0, li))
            elif self.splits[s_]:
                a, b = self.offsets[s_], self.offsets[s_ + 1]
                cw_out.index_add_(0, self.recv_idx[s_], self.recv[a:b])

    def global_rows(self, cw: torch.Tensor) -> torch.Tensor:
        """Full [V, width] matrix of global sums (collective: every rank must call it)."""
        import torch.distributed as td

        g = cw * self.owned.unsqueeze(1).to(cw.dtype)
        cdev = self.ctx._coll_device()
        gc = g.to(cdev)
        td.all_reduce(gc)
        return gc.to(cw.device)


CHAIN_KAPPA = 88.0   # chain cost of one word of the longest document / throughput cost of one entry:
                     # headline day, K = 20: 1.64 ms for 22,721 words vs ~1.1 ms for the other 1.34 M entries


def chain_kappa(K: int = None) -> float:
    """CHAIN_KAPPA at K topics.  The chain costs ~72-76 ns per word at K = 20 and K = 100 alike (a chunk's
    refresh, not its K-wide rows, sets the pace), while an entry's throughput cost grows with K: 0.82 ns
    at K = 20, 2.7 ns at K = 100 (config 5: 245 ms for 90.3 M entries, its 443 k-word chain 33.6 ms,
    r4_strong_emulated.md) -- kappa ~ 88 (20 / K)^0.74.  Unknown K: the K = 20 value."""
    if not K:
        return CHAIN_KAPPA
    return CHAIN_KAPPA * (20.0 / float(K)) ** 0.74


# Per-entry cost of a document by its length, ns at K = 100 (documents of <= 4 | 5-256 | 257-2048 | > 2048
# words): a least-squares fit of 14 measured config-5 shard iterations at N = 2 / 4 / 8 (plus 3.2 ms per
# rank), residual 2.3 ms rms (profiles/r6_strong_emulated.md).  Short documents converge in ~3 sweeps,
# long ones run all 20: entries are not the unit of work, so nnz-balanced cuts left the ranks of the
# month's long documents at 2x the others (38.5 vs 17.1 ms at N = 8).
COST_EDGES = (4, 256, 2048)
COST_NS_K100 = (2.27, 1.30, 1.79, 3.17)
CHAIN_NS_PER_WORD = 72.0   # one-workgroup chain (gs_wsteam / gs_team): ~72 ns per word, K = 20 and 100 alike
SPLIT_CHAIN_NS = 6.0e6     # K > 32: a split document's chain is ~U x sweeps chunk exchanges (443 k words: 6.0 ms)


def doc_costs(lens, K: int = None) -> np.ndarray:
    """Modelled E-step cost (ns) of each document: its entries x the per-entry cost of its length class,
    scaled from K = 100 as an entry's throughput cost scales (~K^0.74, chain_kappa)."""
    lens = np.asarray(lens, np.int64)
    w = np.asarray(COST_NS_K100, np.float64) * ((float(K) / 100.0) ** 0.74 if K else 1.0)
    return lens * w[np.searchsorted(np.asarray(COST_EDGES), lens, side="left")]


def chain_ns(L: int, K: int = None) -> float:
    """Modelled serial chain (ns) of an L-word document: one workgroup's chunk refreshes, or at K > 32 past
    the split threshold the split kernel's exchange-bound chain."""
    t = CHAIN_NS_PER_WORD * float(L)
    if K and K > 32 and L > 2048:
        t = min(t, SPLIT_CHAIN_NS)
    return t


def chain_bounds(doc_ptr: np.ndarray, world: int, kappa: float = None, K: int = None):
    """Chain- and cost-aware contiguous shards.  A rank costs the modelled E-step cost of its documents
    (``doc_costs``: entries weighted by length class); the rank holding the longest document costs that
    document's serial chain (``chain_ns``) plus its other documents.  Candidates: the cost-balanced cut,
    and every split of the other world - 1 ranks between the documents left and right of the longest one
    (a side given no rank shares the longest document's rank); the cheapest wins (largest rank, then the
    largest of the other ranks).  Cost-balanced cuts alone when the chain does not bound the shards
    (chain <= total / world).  ``kappa`` (tests): the chain as kappa x length in entry units, unweighted --
    the round-4 rule."""
    D = len(doc_ptr) - 1
    if world < 2 or D < world:
        return shard_bounds(doc_ptr, world)
    ptr = np.asarray(doc_ptr, np.int64)
    lens = np.diff(ptr)
    if kappa is not None:
        cost = lens.astype(np.float64)
        chain_of = lambda L: kappa * L   # noqa: E731
    else:
        cost = doc_costs(lens, K)
        chain_of = lambda L: chain_ns(L, K)   # noqa: E731
    cptr = np.concatenate([[0.0], np.cumsum(cost)])
    total = float(cptr[-1])
    p = int(np.argmax(lens))
    L = int(lens[p])
    chain = chain_of(L)
    base = shard_bounds(cptr, world)
    if chain <= total / world:
        return base

    def rank_cost(bounds):
        worst, other = 0.0, 0.0
        for a, b in bounds:
            e = float(cptr[b] - cptr[a])
            if a <= p < b:
                worst = max(worst, chain + e - float(cost[p]))
            else:
                worst, other = max(worst, e), max(other, e)
        return worst, other

    cands = [base]
    for kl in range(world):
        kr = world - 1 - kl
        if (kl and p == 0) or (kr and p == D - 1) or kl > p or kr > D - 1 - p:
            continue                    # a rank for a side without (enough) documents
        out = list(shard_bounds(cptr[:p + 1], kl)) if kl else []
        out.append((0 if not kl else p, D if not kr else p + 1))
        if kr:
            sub = cptr[p + 1:] - cptr[p + 1]
            out += [(p + 1 + a, p + 1 + b) for a, b in shard_bounds(sub, kr)]
        cands.append(out)
    return min(cands, key=rank_cost)


def chain_default() -> bool:
    """Chain-aware document shards are the default (ONI_SHARD_CHAIN=0: plain nnz-balanced cuts)."""
    return knobs.get("ONI_SHARD_CHAIN", "1") != "0"


def engine_bounds(doc_ptr: np.ndarray, world: int, K: int = None):
    """The engine's document shards of a corpus split over ``world`` ranks: chain-aware
    (``chain_bounds``) unless ONI_SHARD_CHAIN=0.  The strong-scaling engine (``shard_range``), the
    row-sharded pipeline's corpus builder (corpus/sharded.py) and its resume path all use this rule, so
    a rank's gamma rows and its document names always cover the same documents (``K``: the model's
    topics, which set the chain's relative cost; every caller of one run passes the same K)."""
    return shard_bounds(doc_ptr, world, chain=chain_default(), K=K)


def shard_bounds(doc_ptr: np.ndarray, world: int, chain: bool = False, K: int = None):
    """Contiguous [d0, d1) ranges with ~equal nnz (ties broken toward equal doc counts); ``doc_ptr`` may be
    any cumulative weight (chain_bounds passes the modelled costs).
    ``chain``: ``chain_bounds`` instead (``engine_bounds``, the default rule of the engine's shards)."""
    if chain:
        return chain_bounds(doc_ptr, world, K=K)
    D = len(doc_ptr) - 1
    nnz = doc_ptr[-1]
    if world <= 1 or D == 0:
        return [(0, D)]
    bounds = [0]
    for r in range(1, world):
        target = nnz * r / world
        d = int(np.searchsorted(doc_ptr, target, side="left"))
        d = min(max(d, bounds[-1]), D)
        bounds.append(d)
    bounds.append(D)
    return [(bounds[i], bounds[i + 1]) for i in range(world)]


def init_from_env(expected_world: int = None, backend: str = None, timeout_s: float = 600.0) -> DistContext:
    """Initialise from torchrun env (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if expected_world is not None and expected_world != world and world != 1:
        raise RuntimeError(f"--gpus {expected_world} but WORLD_SIZE={world}")
    if backend is None:
        # ONI_DIST_BACKEND=gloo rehearses several ranks on one GPU (RCCL needs one GPU per rank)
        backend = knobs.get("ONI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available() and backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    elif torch.cuda.is_available():
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    else:
        dev = torch.device("cpu")
    if not knobs.get("ONI_THREADS"):       # an explicit ONI_THREADS: the operator sizes the host
        from ..utils import hostres
        hostres.bind_rank(local, dev)      # the GPU's NUMA node CPUs, a per-rank thread budget
    forced = knobs.get("ONI_DIST_FORCE_GROUP", "0") == "1"
    ctx = DistContext(rank=rank, world_size=world, local_rank=local, device=dev, backend=backend,
                      deterministic=knobs.get("ONI_DIST_DETERMINISTIC", "0") == "1", forced=forced)
    if world > 1 or forced:
        os.environ.setdefault("MASTER_PORT", "29533")
        import torch.distributed as td

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        td.init_process_group(**kw)
        ctx.self_check()
    return ctx
