"""Collectives of the row-sharded pipeline stages (the reference's Spark shuffles / broadcasts / HDFS
part files; ml_ops.sh:57,108).

Everything travels as tensors through the process group's collective device (RCCL device buffers
on the GPU box, host tensors under gloo) -- no pickled objects:

* ``allgather_array`` / ``alltoallv``: variable-length arrays of any dtype (as raw bytes);
* ``first_appearance``: a global string dictionary in first-appearance order (rank order, then each
  rank's local order), hash-partitioned over the ranks as fixed-width integer rows (the Spark job's
  distinct + zipWithIndex, flow_pre_lda.scala) and kept in id-range slices (``DistNameTable``);
* ``fetch_rows`` / ``range_put``: rows of a table held in contiguous row ranges, fetched by the ranks
  that need them (the scorers' model rows, the doc row of an ip) instead of replicated;
* ``write_segments``: every rank writes its own formatted rows at its byte offset of the shared
  output file (the reference's ``part-*`` files concatenated by ``cat`` in part order,
  ml_ops.sh:59-62,110-115);
* ``merge_sorted_rows``: the ``sortByKey`` range-partition shuffle of the scored rows
  (flow_post_lda.scala:245-248, dns_post_lda.scala:326-331): a global stable ascending order of every
  rank's survivors, the rows moved so rank r holds the r-th contiguous slice, then one segment write;
* ``chain``: a rank-order sequential fold (0 + part_0, then + part_1, ...) -- a reduction whose
  result does not depend on the number of ranks (the bitwise test mode of the sharded pipeline).

With one rank (or no initialised process group) every helper degenerates to the local operation.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


def _active(ctx) -> bool:
    return ctx is not None and getattr(ctx, "initialized", False)


def world(ctx) -> int:
    return ctx.world_size if _active(ctx) else 1


def rank(ctx) -> int:
    return ctx.rank if _active(ctx) else 0


def _dev(ctx):
    return ctx._coll_device()


def allgather_sizes(ctx, n: int) -> List[int]:
    if not _active(ctx):
        return [int(n)]
    import torch.distributed as td
    t = torch.tensor([int(n)], dtype=torch.int64, device=_dev(ctx))
    out = [torch.zeros_like(t) for _ in range(ctx.world_size)]
    td.all_gather(out, t)
    return [int(x.item()) for x in out]


def allreduce_max_int(ctx, v: int) -> int:
    if not _active(ctx):
        return int(v)
    import torch.distributed as td
    t = torch.tensor([int(v)], dtype=torch.int64, device=_dev(ctx))
    td.all_reduce(t, op=td.ReduceOp.MAX)
    return int(t.item())


def _as_bytes(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a)
    return a.reshape(-1).view(np.uint8)


def allgather_array(ctx, a: np.ndarray) -> List[np.ndarray]:
    """Every rank's array (same dtype and trailing shape, any length), in rank order."""
    a = np.ascontiguousarray(a)
    if not _active(ctx):
        return [a]
    import torch.distributed as td
    tail = a.shape[1:]
    sizes = allgather_sizes(ctx, a.shape[0])
    row_bytes = a.dtype.itemsize * int(np.prod(tail, dtype=np.int64))
    mx = max(max(sizes), 1) * row_bytes
    buf = torch.zeros(mx, dtype=torch.uint8, device=_dev(ctx))
    b = _as_bytes(a)
    if b.size:
        buf[: b.size] = torch.from_numpy(b).to(buf.device)
    outs = [torch.empty_like(buf) for _ in range(ctx.world_size)]
    td.all_gather(outs, buf)
    res = []
    for o, n in zip(outs, sizes):
        raw = o[: n * row_bytes].cpu().numpy()
        res.append(raw.view(a.dtype).reshape((n,) + tail) if n else np.zeros((0,) + tail, a.dtype))
    return res


def alltoallv(ctx, parts: Sequence[np.ndarray]) -> List[np.ndarray]:
    """parts[s] goes to rank s; returns what every rank sent here, in rank order."""
    if not _active(ctx):
        return [np.ascontiguousarray(parts[0])]
    import torch.distributed as td
    N = ctx.world_size
    assert len(parts) == N
    dt = parts[0].dtype
    tail = parts[0].shape[1:]
    row_bytes = dt.itemsize * int(np.prod(tail, dtype=np.int64))
    send_rows = torch.tensor([p.shape[0] for p in parts], dtype=torch.int64, device=_dev(ctx))
    recv_rows = torch.empty_like(send_rows)
    td.all_to_all_single(recv_rows, send_rows)
    send_b = [int(n) * row_bytes for n in send_rows.cpu().tolist()]
    recv_n = recv_rows.cpu().tolist()
    recv_b = [int(n) * row_bytes for n in recv_n]
    flat = np.concatenate([_as_bytes(np.asarray(p, dt)) for p in parts]) if sum(send_b) else np.zeros(0, np.uint8)
    sbuf = torch.from_numpy(flat).to(_dev(ctx)) if flat.size else torch.zeros(0, dtype=torch.uint8, device=_dev(ctx))
    rbuf = torch.empty(sum(recv_b), dtype=torch.uint8, device=_dev(ctx))
    td.all_to_all_single(rbuf, sbuf, recv_b, send_b)
    raw = rbuf.cpu().numpy()
    out, off = [], 0
    for n, nb in zip(recv_n, recv_b):
        out.append(raw[off:off + nb].view(dt).reshape((int(n),) + tail) if nb else np.zeros((0,) + tail, dt))
        off += nb
    return out


def broadcast_array(ctx, a: Optional[np.ndarray], src: int = 0, dtype=None) -> np.ndarray:
    """Rank ``src``'s array on every rank (``a`` may be None elsewhere; ``dtype`` must then be given)."""
    if not _active(ctx):
        return a
    import torch.distributed as td
    meta = torch.zeros(8, dtype=torch.int64, device=_dev(ctx))
    if ctx.rank == src:
        a = np.ascontiguousarray(a)
        meta[0] = a.ndim
        meta[1: 1 + a.ndim] = torch.tensor(a.shape, dtype=torch.int64)
    td.broadcast(meta, src=src)
    nd = int(meta[0])
    shape = tuple(int(x) for x in meta[1:1 + nd].tolist())
    dt = a.dtype if ctx.rank == src else np.dtype(dtype)
    nbytes = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
    buf = torch.empty(nbytes, dtype=torch.uint8, device=_dev(ctx))
    if ctx.rank == src and nbytes:
        buf.copy_(torch.from_numpy(_as_bytes(a)).to(buf.device))
    if nbytes:
        td.broadcast(buf, src=src)
    return buf.cpu().numpy().view(dt).reshape(shape)


def chain(ctx, fold, carry0: np.ndarray) -> np.ndarray:
    """Rank-order sequential fold: rank 0 computes fold(carry0), rank r computes fold(result of r - 1);
    the last rank's result is returned on every rank.  ``fold`` continues a sequential sum from the
    carry, so the result is bitwise what one process folding all parts in order computes."""
    if not _active(ctx):
        return fold(carry0)
    import torch.distributed as td
    r, N = ctx.rank, ctx.world_size
    carry = np.ascontiguousarray(carry0)
    if r > 0:
        t = torch.empty(carry.size, dtype=torch.float64, device=_dev(ctx))
        td.recv(t, src=r - 1)
        carry = t.cpu().numpy().reshape(carry0.shape)
    out = np.ascontiguousarray(fold(carry), dtype=np.float64)
    if r < N - 1:
        td.send(torch.from_numpy(out.reshape(-1)).to(_dev(ctx)), dst=r + 1)
    return broadcast_array(ctx, out if r == N - 1 else None, src=N - 1, dtype=np.float64)


# ------------------------------------------------------------------------------------ dictionaries
class NameTable:
    """Strings as a fixed-width byte matrix (NUL padded): decoded only where text is needed."""

    def __init__(self, mat: np.ndarray):
        self.mat = np.ascontiguousarray(mat, np.uint8)

    def __len__(self):
        return self.mat.shape[0]

    def take(self, ids) -> List[str]:
        ids = np.asarray(ids, np.int64)
        if self.mat.shape[1] == 0:
            return [""] * ids.size
        s = self.mat[ids].view(f"S{self.mat.shape[1]}").reshape(-1)
        return np.char.decode(s, "utf-8", errors="surrogateescape").tolist()

    def all(self) -> List[str]:
        return self.take(np.arange(len(self)))


def pack_names(data: np.ndarray, off: np.ndarray, width: Optional[int] = None) -> np.ndarray:
    """(bytes, offsets [n + 1]) -> [n, width] uint8, NUL padded; width = max length rounded up to 8."""
    off = np.asarray(off, np.int64)
    lens = np.diff(off)
    n = lens.size
    w = int(lens.max()) if n else 0
    W = width if width is not None else max(8, -(-w // 8) * 8)
    if w > W:
        raise ValueError("name longer than the packed width")
    mat = np.zeros((n, W), np.uint8)
    if n and off[-1] > off[0]:
        rows = np.repeat(np.arange(n, dtype=np.int64), lens)
        cols = np.arange(int(off[-1] - off[0]), dtype=np.int64) - np.repeat(off[:-1] - off[0], lens)
        mat[rows, cols] = np.frombuffer(memoryview(data), np.uint8)[off[0]:off[-1]]
    return mat


def names_to_bytes(names: Sequence[str]):
    enc = [s.encode("utf-8", errors="surrogateescape") for s in names]
    off = np.zeros(len(enc) + 1, np.int64)
    if enc:
        np.cumsum([len(b) for b in enc], out=off[1:])
    return np.frombuffer(b"".join(enc), np.uint8), off


def range_starts(total: int, n: int) -> List[int]:
    """Range partition of ids [0, total) over n ranks: rank s owns [starts[s], starts[s + 1])."""
    return [int(total) * s // n for s in range(n + 1)]


def fetch_rows(ctx, local: np.ndarray, starts: Sequence[int], query) -> np.ndarray:
    """Rows of a table held in contiguous row ranges (rank s keeps global rows [starts[s], starts[s + 1])
    as ``local``), for the global ids ``query`` (any order, repeats allowed; -1: a zero row).  Collective:
    every rank asks only for the rows it needs (two ``alltoallv``), nothing is replicated."""
    local = np.ascontiguousarray(local)
    q = np.asarray(query, np.int64).reshape(-1)
    valid = q >= 0
    uq, inv = np.unique(q[valid], return_inverse=True)
    N, r = world(ctx), rank(ctx)
    st = np.asarray(starts, np.int64)
    if not _active(ctx):
        got = local[uq - st[0]]
    else:
        owner = np.searchsorted(st, uq, side="right") - 1
        cuts = np.searchsorted(owner, np.arange(N + 1), side="left")
        req = alltoallv(ctx, [uq[cuts[d]:cuts[d + 1]] for d in range(N)])
        if any(x.size and (x.min() < st[r] or x.max() >= st[r + 1]) for x in req):
            raise IndexError("fetch_rows: a request outside this rank's rows")
        resp = alltoallv(ctx, [local[x - st[r]] for x in req])
        got = np.concatenate(resp) if resp else local[:0]
    out = np.zeros((q.size,) + local.shape[1:], local.dtype)
    if uq.size:
        out[valid] = got[inv]
    return out


def range_put(ctx, ids, rows: np.ndarray, total: int, fill=0) -> np.ndarray:
    """(id, row) pairs of every rank -> the rank owning each id's range (``range_starts(total, N)``);
    returns this rank's slice [starts[r], starts[r + 1]) (ids never sent keep ``fill``)."""
    ids = np.asarray(ids, np.int64).reshape(-1)
    rows = np.ascontiguousarray(rows)
    N, r = world(ctx), rank(ctx)
    st = range_starts(total, N)
    o = np.argsort(ids, kind="stable")
    ids_s, rows_s = ids[o], rows[o]
    cuts = np.searchsorted(ids_s, np.asarray(st, np.int64), side="left")
    if _active(ctx):
        rid = np.concatenate(alltoallv(ctx, [ids_s[cuts[d]:cuts[d + 1]] for d in range(N)]))
        rrow = np.concatenate(alltoallv(ctx, [rows_s[cuts[d]:cuts[d + 1]] for d in range(N)]))
    else:
        rid, rrow = ids_s, rows_s
    lo, hi = st[r], st[r + 1]
    out = np.full((hi - lo,) + rows.shape[1:], fill, rows.dtype)
    if rid.size:
        out[rid - lo] = rrow
    return out


class DistNameTable:
    """A global dictionary (ids 0 .. total - 1) held in range slices: rank r keeps the names of ids
    [total r / N, total (r + 1) / N) as fixed-width byte rows.  ``take`` is collective (``fetch_rows``):
    a rank receives only the names it asks for."""

    def __init__(self, ctx, mat: np.ndarray, lens: np.ndarray, total: int):
        self.ctx, self.total = ctx, int(total)
        self.mat = np.ascontiguousarray(mat, np.uint8)
        self.lens = np.ascontiguousarray(lens, np.int64)
        self.starts = range_starts(self.total, world(ctx))

    def __len__(self):
        return self.total

    def all(self) -> List[str]:
        """Every name on every rank (collective; for small dictionaries, e.g. DNS query types)."""
        return self.take(np.arange(self.total, dtype=np.int64))

    def take(self, ids) -> List[str]:
        ids = np.asarray(ids, np.int64).reshape(-1)
        rows = fetch_rows(self.ctx, np.concatenate([self.mat.view(np.int64).reshape(self.mat.shape[0], -1),
                                                    self.lens[:, None]], 1), self.starts, ids)
        W = self.mat.shape[1]
        m = np.ascontiguousarray(rows[:, :W // 8]).view(np.uint8).reshape(ids.size, W)
        ln = rows[:, W // 8]
        out = []
        for i in range(ids.size):
            out.append(bytes(m[i, :ln[i]]).decode("utf-8", errors="surrogateescape"))
        return out


class DistDict:
    """name -> int64 value over the ranks, hash-partitioned by name: rank hash(name) mod N keeps the
    entries of its names.  Where several entries share a name the largest value wins -- the map the
    Scala scorers build with ``collectAsMap`` over word_results.csv rows (later rows win,
    flow_post_lda.scala:107-123).  Construction and ``lookup`` are collective; nothing is replicated."""

    def __init__(self, ctx, names: Sequence[str], values):
        self.ctx = ctx
        N = world(ctx)
        data, off = names_to_bytes(names)
        lens = np.diff(off)
        self.W = max(8, -(-allreduce_max_int(ctx, int(lens.max()) if lens.size else 0) // 8) * 8)
        key = self._key(data, off)
        vals = np.asarray(values, np.int64).reshape(-1, 1)
        owner = self._owner(key)
        o = np.argsort(owner, kind="stable")
        cuts = np.searchsorted(owner[o], np.arange(N + 1), side="left")
        send = np.concatenate([key, vals], 1)[o]
        recv = alltoallv(ctx, [send[cuts[d]:cuts[d + 1]] for d in range(N)]) if N > 1 else [send]
        allr = np.concatenate(recv) if recv else send[:0]
        if allr.shape[0]:
            u, inv = unique_rows(np.ascontiguousarray(allr[:, :-1]))
            v = np.full(u.shape[0], -1, np.int64)
            np.maximum.at(v, inv, allr[:, -1])
            self.keys, self.vals = u, v
        else:
            self.keys, self.vals = allr[:, :-1], np.zeros(0, np.int64)

    def _key(self, data, off) -> np.ndarray:
        off = np.asarray(off, np.int64)
        lens = np.diff(off)
        mat = pack_names(data, off, self.W)
        return np.concatenate([mat.view(np.int64).reshape(lens.size, self.W // 8), lens[:, None]], 1)

    def _owner(self, key) -> np.ndarray:
        N = world(self.ctx)
        return (_row_hash(key) % np.uint64(N)).astype(np.int64) if N > 1 else np.zeros(key.shape[0], np.int64)

    def lookup(self, names: Sequence[str]) -> np.ndarray:
        """Value of every name (-1: absent).  Collective."""
        N = world(self.ctx)
        data, off = names_to_bytes(names)
        lens = np.diff(off)
        fits = lens <= self.W                    # longer names cannot be keys
        idx = np.flatnonzero(fits)
        sub_off = np.concatenate([[0], np.cumsum(lens[idx])]).astype(np.int64)
        raw = np.frombuffer(memoryview(data), np.uint8) if len(data) else np.zeros(0, np.uint8)
        sub = raw if fits.all() else raw[np.repeat(fits, lens)]
        key = self._key(sub, sub_off)
        owner = self._owner(key)
        o = np.argsort(owner, kind="stable")
        cuts = np.searchsorted(owner[o], np.arange(N + 1), side="left")
        q = key[o]
        recv = alltoallv(self.ctx, [q[cuts[d]:cuts[d + 1]] for d in range(N)]) if N > 1 else [q]
        rsz = [x.shape[0] for x in recv]
        allq = np.concatenate(recv) if recv else q[:0]
        ans = np.full(allq.shape[0], -1, np.int64)
        if allq.shape[0] and self.keys.shape[0]:
            _, inv = unique_rows(np.ascontiguousarray(np.concatenate([self.keys, allq])))
            val_u = np.full(int(inv.max()) + 1, -1, np.int64)
            val_u[inv[:self.keys.shape[0]]] = self.vals
            ans = val_u[inv[self.keys.shape[0]:]]
        rc = np.concatenate([[0], np.cumsum(rsz)])
        back = alltoallv(self.ctx, [ans[rc[d]:rc[d + 1]] for d in range(N)]) if N > 1 else [ans]
        got = np.empty(idx.size, np.int64)
        got[o] = np.concatenate(back) if back else np.zeros(0, np.int64)
        out = np.full(lens.size, -1, np.int64)
        out[idx] = got
        return out


def _row_hash(rows64: np.ndarray) -> np.ndarray:
    """A 64-bit mix of each int64 row (the owner of a name in the hash-partitioned dictionary)."""
    h = np.zeros(rows64.shape[0], np.uint64)
    with np.errstate(over="ignore"):
        for j in range(rows64.shape[1]):
            h = (h ^ rows64[:, j].view(np.uint64)) * np.uint64(0x9E3779B97F4A7C15)
            h ^= h >> np.uint64(29)
    return h


def unique_rows(rows64: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """(distinct rows, inverse) of an int64 [n, c] array, rows grouped by a 64-bit hash (one argsort of
    n keys) and checked for equality within each hash run; a run that mixes rows (a hash collision)
    falls back to a lexicographic sort.  (torch.unique(dim=0) on the host took 13.8 s for 3 M rows of
    3 columns here, this 0.5 s: the 8-rank config-5 flow_pre spent minutes in it, profiles/r4_config5.md.)"""
    n = rows64.shape[0]
    h = _row_hash(rows64)
    o = np.argsort(h, kind="stable")
    hs, ks = h[o], rows64[o]
    new_h = np.empty(n, bool)
    new_h[0] = True
    np.not_equal(hs[1:], hs[:-1], out=new_h[1:])
    new_r = np.empty(n, bool)
    new_r[0] = True
    np.any(ks[1:] != ks[:-1], axis=1, out=new_r[1:])
    if np.any(new_r & ~new_h):          # equal hashes, different rows: sort the rows themselves
        o = np.lexsort(rows64.T[::-1])
        ks = rows64[o]
        new_r[1:] = np.any(ks[1:] != ks[:-1], axis=1)
    gid = np.cumsum(new_r) - 1
    inv = np.empty(n, np.int64)
    inv[o] = gid
    return ks[new_r], inv


def first_appearance(ctx, data: np.ndarray, off: np.ndarray) -> Tuple[DistNameTable, np.ndarray]:
    """Global dictionary of every rank's local dictionary (each in local first-appearance order): ids in
    order of first appearance over the ranks' rows in rank order -- the single-process dictionary of
    the concatenated input.  Returns (global names, local id -> global id).

    Hash-partitioned, nothing replicated (the Spark job's distinct + zipWithIndex, not a driver-side
    collect): every name goes, with its global position (lower ranks' names first, then local order), to
    the rank owning hash(name); owners merge duplicates keeping the minimum position; each first
    position goes to the rank whose position range holds it, where a prefix count over the ranks gives
    its global id; the ids travel back to the owners and on to every sender; the names land in range
    slices by id (``DistNameTable``).  Rows carry the name length, so names that differ only by
    trailing NUL bytes stay distinct."""
    N, r = world(ctx), rank(ctx)
    off = np.asarray(off, np.int64)
    lens = np.diff(off)
    n = lens.size
    w = allreduce_max_int(ctx, int(lens.max()) if n else 0)
    W = max(8, -(-w // 8) * 8)
    mat = pack_names(data, off, W)
    sizes = allgather_sizes(ctx, n)
    base = sum(sizes[:r])
    key = np.concatenate([mat.view(np.int64).reshape(n, W // 8), lens[:, None]], 1)     # [n, W/8 + 1]
    pos = base + np.arange(n, dtype=np.int64)
    owner = (_row_hash(key) % np.uint64(N)).astype(np.int64) if N > 1 else np.zeros(n, np.int64)
    o = np.argsort(owner, kind="stable")
    cuts = np.searchsorted(owner[o], np.arange(N + 1), side="left")
    send = np.concatenate([key, pos[:, None]], 1)[o]
    recv = alltoallv(ctx, [send[cuts[d]:cuts[d + 1]] for d in range(N)]) if N > 1 else [send]
    rsz = [x.shape[0] for x in recv]
    allr = np.concatenate(recv) if recv else send[:0]
    # ---- owner: distinct names, minimum position
    if allr.shape[0]:
        uniq, inv = unique_rows(np.ascontiguousarray(allr[:, :-1]))
        minpos = np.full(uniq.shape[0], np.iinfo(np.int64).max, np.int64)
        np.minimum.at(minpos, inv, allr[:, -1])
    else:
        uniq, inv, minpos = allr[:, :-1], np.zeros(0, np.int64), np.zeros(0, np.int64)
    # ---- global ids: first positions counted in position order, across the ranks' position ranges
    pstarts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    powner = np.searchsorted(pstarts, minpos, side="right") - 1
    po = np.argsort(powner, kind="stable")
    pcuts = np.searchsorted(powner[po], np.arange(N + 1), side="left")
    firsts = alltoallv(ctx, [minpos[po][pcuts[d]:pcuts[d + 1]] for d in range(N)]) if N > 1 else [minpos]
    fl = np.concatenate(firsts) if firsts else minpos
    cnt = allgather_sizes(ctx, fl.size)
    total = int(sum(cnt))
    rank_in = np.empty(fl.size, np.int64)
    rank_in[np.argsort(fl, kind="stable")] = np.arange(fl.size, dtype=np.int64)
    gid_fl = sum(cnt[:r]) + rank_in
    fcuts = np.concatenate([[0], np.cumsum([x.size for x in firsts])])
    back = alltoallv(ctx, [gid_fl[fcuts[d]:fcuts[d + 1]] for d in range(N)]) if N > 1 else [gid_fl]
    gid_u = np.empty(minpos.size, np.int64)
    gid_u[po] = np.concatenate(back) if back else np.zeros(0, np.int64)
    # ---- every sender's names get their ids (same order as sent)
    gid_rows = gid_u[inv] if inv.size else np.zeros(0, np.int64)
    rcuts = np.concatenate([[0], np.cumsum(rsz)])
    mine = alltoallv(ctx, [gid_rows[rcuts[d]:rcuts[d + 1]] for d in range(N)]) if N > 1 else [gid_rows]
    lmap = np.empty(n, np.int64)
    lmap[o] = np.concatenate(mine) if mine else np.zeros(0, np.int64)
    # ---- the names by id range
    rows = range_put(ctx, gid_u, np.ascontiguousarray(uniq), total) if total else uniq[:0]
    tab = np.ascontiguousarray(rows[:, :W // 8]).view(np.uint8).reshape(rows.shape[0], W)
    return DistNameTable(ctx, tab, rows[:, W // 8], total), lmap


# ------------------------------------------------------------------------------------ file output
def write_segments(ctx, path: str, segs: Sequence[np.ndarray]) -> int:
    """Shared output file = segment 0 of ranks 0..N-1, then segment 1 of ranks 0..N-1, ...  (every
    rank passes the same number of uint8 segments).  Rank 0 creates the file at its final size,
    then every rank pwrite()s its segments at their offsets.  Returns the file size."""
    segs = [np.ascontiguousarray(s, np.uint8).reshape(-1) for s in segs]
    N = world(ctx)
    mine = np.asarray([s.size for s in segs], np.int64)
    allsz = np.stack(allgather_array(ctx, mine)) if N > 1 else mine[None, :]    # [N, S]
    order = allsz.T.reshape(-1)                                                   # segment-major
    offs = np.concatenate([[0], np.cumsum(order)])
    total = int(offs[-1])
    r = rank(ctx)
    if r == 0:
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        os.ftruncate(fd, total)
        os.close(fd)
    if N > 1:
        ctx.barrier()
    fd = os.open(path, os.O_WRONLY)
    try:
        for s_, seg in enumerate(segs):
            o = int(offs[s_ * N + r])
            mv = memoryview(seg)
            while mv.nbytes:
                k = os.pwrite(fd, mv, o)
                mv, o = mv[k:], o + k
    finally:
        os.close(fd)
    if N > 1:
        ctx.barrier()
    return total


def merge_sorted_rows(ctx, keys: np.ndarray, text: np.ndarray, row_ends: np.ndarray, path: str) -> int:
    """Write every rank's rows into one file in global ascending key order, ties in rank order then
    local order (one process's stable sort over the rows in input order).  ``keys`` (float64) are
    this rank's row keys, already ascending (stable); ``text`` / ``row_ends`` their formatted lines.
    Returns the number of rows in the file."""
    from ..ops import native
    keys = np.ascontiguousarray(keys, np.float64)
    N, r = world(ctx), rank(ctx)
    if not _active(ctx):
        write_segments(ctx, path, [text])
        return int(keys.size)
    all_keys = allgather_array(ctx, keys)
    total = sum(k.size for k in all_keys)
    pos = np.arange(keys.size, dtype=np.int64)
    for s_, ks in enumerate(all_keys):
        if s_ < r:
            pos += np.searchsorted(ks, keys, side="right")
        elif s_ > r:
            pos += np.searchsorted(ks, keys, side="left")
    # destination: rank d holds global rows [total d / N, total (d + 1) / N)
    bounds = np.asarray([total * d // N for d in range(N + 1)], np.int64)
    dest = np.searchsorted(bounds, pos, side="right") - 1
    ends = np.asarray(row_ends, np.int64)
    starts = np.concatenate([[0], ends[:-1]]) if ends.size else ends
    cut_rows = np.searchsorted(dest, np.arange(N + 1), side="left")
    cut_bytes = np.concatenate([[0], ends])[cut_rows]
    t_parts = [text[cut_bytes[d]:cut_bytes[d + 1]] for d in range(N)]
    meta = np.stack([pos, ends - starts], 1) if keys.size else np.zeros((0, 2), np.int64)
    m_parts = [meta[cut_rows[d]:cut_rows[d + 1]] for d in range(N)]
    t_recv = alltoallv(ctx, t_parts)
    m_recv = alltoallv(ctx, m_parts)
    buf = np.concatenate(t_recv) if t_recv else np.zeros(0, np.uint8)
    m = np.concatenate(m_recv) if m_recv else np.zeros((0, 2), np.int64)
    lens = m[:, 1]
    st = np.concatenate([[0], np.cumsum(lens)[:-1]]) if lens.size else lens
    o = np.argsort(m[:, 0], kind="stable")
    out = native.lib().concat_spans(buf, st[o], lens[o]) if lens.size else np.zeros(0, np.uint8)
    write_segments(ctx, path, [out])
    return total


def concat_part_files(ctx, path: str, part: str) -> int:
    """Every rank's ``part`` file -> ``path`` in rank order (the reference's ``cat part-*``), then the
    parts are removed.  Collective.  Returns the file size."""
    size = os.path.getsize(part) if os.path.exists(part) else 0
    sizes = allgather_sizes(ctx, size)
    r, N = rank(ctx), world(ctx)
    off, total = sum(sizes[:r]), sum(sizes)
    if r == 0:
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        os.ftruncate(fd, total)
        os.close(fd)
    if N > 1:
        ctx.barrier()
    if size:
        fi = os.open(part, os.O_RDONLY)
        fo = os.open(path, os.O_WRONLY)
        try:
            done = 0
            while done < size:
                try:
                    k = os.copy_file_range(fi, fo, size - done, done, off + done)
                except OSError:
                    k = os.pwrite(fo, os.pread(fi, min(size - done, 1 << 26), done), off + done)
                if k <= 0:
                    raise OSError(f"short copy of {part} into {path}")
                done += k
        finally:
            os.close(fi)
            os.close(fo)
    if N > 1:
        ctx.barrier()
    if os.path.exists(part):
        os.unlink(part)
    return total
