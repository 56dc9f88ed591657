"""Process-group context: one process per GPU, RCCL over xGMI (torch backend "nccl").

Replaces the reference's MPI layer (`mpiexec -n 20 -f machinefile ./lda est ...`,
ml_ops.sh:80):

* documents are sharded CONTIGUOUSLY and balanced by nnz (not doc count), so the
  per-rank gamma blocks concatenate in corpus order exactly like lda-c's
  per-worker <rank>.gamma files combined into final.gamma (README.md:121);
* per EM iteration the only collective is one all-reduce of the flat class_word
  buffer [V x KS] f32 plus a 2-scalar f64 all-reduce (likelihood, alpha ss) —
  ring all-reduce over the 7 xGMI links of a node, K*V*4 bytes;
* the CPU test path runs the same code over gloo.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def initialized(self) -> bool:
        return self.world_size > 1 and torch.distributed.is_initialized()

    # -------------------------------------------------------------- sharding
    def shard_range(self, corpus):
        return shard_bounds(corpus.doc_ptr, self.world_size)[self.rank]

    # ----------------------------------------------------------- collectives
    def allreduce_suffstats(self, cw: torch.Tensor, scalars: torch.Tensor) -> torch.Tensor:
        if not self.initialized:
            return scalars
        import torch.distributed as td

        work = td.all_reduce(scalars, async_op=True)
        td.all_reduce(cw)
        work.wait()
        return scalars

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


def shard_bounds(doc_ptr: np.ndarray, world: int):
    """Contiguous [d0, d1) ranges with ~equal nnz (ties broken toward equal doc counts)."""
    D = len(doc_ptr) - 1
    nnz = int(doc_ptr[-1])
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
        backend = os.environ.get("ONI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available() and backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    elif torch.cuda.is_available():
        dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    else:
        dev = torch.device("cpu")
    ctx = DistContext(rank=rank, world_size=world, local_rank=local, device=dev, backend=backend)
    if world > 1:
        import torch.distributed as td

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(backend=backend, rank=rank, world_size=world,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        td.init_process_group(**kw)
    return ctx
