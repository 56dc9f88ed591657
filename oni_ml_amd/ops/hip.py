"""Loader + validated launch wrappers for the gfx950 HIP kernels (`_onihip`).

Every wrapper checks dtype / device / contiguity / shape on the host before it
hands raw addresses to the kernel (a wrong shape on a hand-written kernel can
fault the whole GPU), then launches on torch's current stream so the launch is
ordered with torch work and capturable in a hipGraph.

On a machine with a GPU the extension is mandatory: :func:`lib` raises if it
cannot be imported instead of silently falling back to eager torch.
"""
from __future__ import annotations

import importlib
import os
import sys
from typing import Optional

import torch

_LIB = None
_ERR = None


def _import():
    global _LIB, _ERR
    if _LIB is not None or _ERR is not None:
        return
    try:
        here = os.path.join(os.path.dirname(os.path.dirname(__file__)), "_lib")
        if here not in sys.path:
            sys.path.insert(0, here)
        _LIB = importlib.import_module("_onihip")
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e


def available() -> bool:
    _import()
    return _LIB is not None and torch.cuda.is_available()


def lib():
    """Return the extension module; raise loudly if it is missing."""
    _import()
    if _LIB is None:
        raise RuntimeError(
            "oni_ml_amd HIP extension (_onihip) is not built or failed to load: "
            f"{_ERR!r}. Run `python -m oni_ml_amd._build` (needs hipcc, gfx950)."
        )
    return _LIB


_EXP = None


def exp_lib():
    """The experimental kernels' module (`_onihip_exp`: variants measured not faster, loaded only when a
    caller asks for one -- never by ml_ops); raises loudly if it is missing."""
    global _EXP
    if _EXP is None:
        lib()
        try:
            _EXP = importlib.import_module("_onihip_exp")
        except Exception as e:  # pragma: no cover - depends on build state
            raise RuntimeError(f"oni_ml_amd experimental HIP extension (_onihip_exp) failed to load: {e!r}. "
                               "It is built only on request: `python -m oni_ml_amd._build exp`.") from e
    return _EXP


def exp_available() -> bool:
    """Whether the opt-in experimental module was built (its tests skip otherwise)."""
    import glob
    return bool(glob.glob(os.path.join(os.path.dirname(os.path.dirname(__file__)), "_lib", "_onihip_exp*.so")))


def compiled_ks():
    return list(lib().compiled_ks())


def padded_topics(K: int) -> int:
    """Smallest compiled row stride >= K (multiple of 4)."""
    for ks in (8, 12, 16, 20, 24, 32, 52, 64, 100, 128):
        if ks >= K:
            return ks
    raise ValueError(f"K={K} exceeds the largest compiled topic count (128)")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _chk(t: torch.Tensor, dtype, name, shape=None, device=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_cuda:
        raise ValueError(f"{name}: must be a GPU tensor")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name}: shape {tuple(t.shape)} != {tuple(shape)}")
    return t.data_ptr()


PARAM_COUNT = 8      # device parameter block (csrc/hip/kernels.h kParamCount)
PARAM_DONE = 4       # params[PARAM_DONE] != 0: the EM loop converged, kernels skip
HIST_COLS = 6        # em_control history row: likelihood, conv, alpha, VAR_MAX_ITER, alpha_ss, -


def _params_ptr(params, dev) -> int:
    return 0 if params is None else _chk(params, torch.float64, "params", (PARAM_COUNT,), dev)


def _gate_ptr(gate, dev) -> int:
    """Pointer to a float64 flag (e.g. params[PARAM_DONE:PARAM_DONE+1]) or 0."""
    return 0 if gate is None else _chk(gate, torch.float64, "gate", (1,), dev)


def argsort_desc_stable(keys):
    """np.argsort(-keys, kind="stable") for non-negative integer keys, as numpy's O(n) radix sort on
    16-bit digits (one pass below 2^16, two below 2^32): the length plans are inside the engine
    setup, which bench.py's to-convergence clock includes (4x faster on 124 k document lengths)."""
    import numpy as np
    k = np.asarray(keys, np.int64)
    if k.size == 0:
        return np.zeros(0, np.int64)
    m = int(k.max())
    if int(k.min()) < 0 or m >= 1 << 32:
        return np.argsort(-k, kind="stable")
    r = m - k
    if m < 1 << 16:
        return np.argsort(r.astype(np.uint16), kind="stable")
    o = np.argsort((r & 0xFFFF).astype(np.uint16), kind="stable")
    return o[np.argsort((r[o] >> 16).astype(np.uint16), kind="stable")]


class SuffPlan:
    """Word order for the single-launch suff-stats kernel (gs_suff64): [heavy | medium | light] (heavy first).

    ``words``: restrict the plan to these word ids (a sub-plan; several sub-plans must together
    cover the vocabulary, since every word's class_word row is written by exactly one launch)."""
    HEAVY, LIGHT = 1024, 64

    def __init__(self, word_len, device, words=None):
        import numpy as np
        wl = np.asarray(word_len)
        ids = np.arange(wl.size, dtype=np.int64) if words is None else np.asarray(words, np.int64)
        if ids.size and (ids.min() < 0 or ids.max() >= wl.size):
            raise ValueError("suff sub-plan word ids out of range")
        self.covers_all = words is None
        order = ids[argsort_desc_stable(wl[ids])].astype(np.int32)
        L = wl[order]
        self.n_heavy = int((L > self.HEAVY).sum())
        self.n_medium = int(((L > self.LIGHT) & (L <= self.HEAVY)).sum())
        self.n_light = int((L <= self.LIGHT).sum())
        self.order = torch.from_numpy(order).to(device)
        self.n_blocks = int(lib().suff_fused_blocks(self.n_heavy, self.n_medium, self.n_light))


def _scalar_slice(scalars, D, dev):
    if scalars is None:
        return 0, 0, 0, 0
    lik, ass, lo, hi = scalars
    if not 0 <= lo <= hi <= D:
        raise ValueError(f"scalar slice [{lo}, {hi}) outside [0, {D}]")
    return (_chk(lik, torch.float64, "lik", (D,), dev), _chk(ass, torch.float64, "alpha_ss", (D,), dev),
            int(lo), int(hi))


def rows_accumulate(rows, ptr, src, own, recv, out):
    """out[rows[i]] = 0 + sum over j in [ptr[i], ptr[i+1]) of (own[rows[i]] if src[j] < 0 else recv[src[j]]),
    fp64, in j order (parallel/dist.py VocabExchange.accumulate)."""
    dev = out.device
    V, W = out.shape
    n = rows.numel()
    if n == 0:
        return
    # ptr / src are built and bounds-checked once on the host (VocabExchange.__init__)
    lib().rows_accumulate(_chk(rows, torch.int32, "rows", (n,), dev), _chk(ptr, torch.int32, "ptr", (n + 1,), dev),
                          _chk(src, torch.int32, "src", None, dev), _chk(own, torch.float64, "own", (V, W), dev),
                          _chk(recv, torch.float64, "recv", None, dev), _chk(out, torch.float64, "out", (V, W), dev),
                          int(n), int(W), _stream())


def init_random_ss(cw, K, seed):
    """cw [V, KS] float64 <- lda-c random start 1/V + u(seed, k V + w) (native ``random_ss`` bits)."""
    V, KS = cw.shape
    lib().init_random_ss(_chk(cw, torch.float64, "cw", (V, KS), cw.device), int(V), int(K), int(KS),
                         int(seed) & 0xFFFFFFFFFFFFFFFF, _stream())


def log_beta_t(cw, class_total, K: int, floor: float, out=None):
    """[K, V] float64 log(cw[:, k]) - log(class_total[k]) (``floor`` where cw == 0) of a [V, KS] class_word: the
    saved log beta in file order (csrc/hip/reduce.hip log_beta_t_kernel; bitwise torch's transpose / log / where)."""
    dev = cw.device
    V, KS = cw.shape
    if not (0 < K <= KS):
        raise ValueError(f"log_beta_t: K={K} outside 1..{KS}")
    p_cw = _chk(cw, torch.float64, "cw", (V, KS), dev)
    p_ct = _chk(class_total, torch.float64, "class_total", None, dev)
    if class_total.numel() < K:
        raise ValueError(f"log_beta_t: class_total holds {class_total.numel()} < K = {K} values")
    if out is None:
        out = torch.empty((K, V), dtype=torch.float64, device=dev)
    p_out = _chk(out, torch.float64, "out", (K, V), dev)
    lib().log_beta_t(p_cw, int(V), int(K), int(KS), p_ct, float(floor), p_out, _stream())
    return out


def colsum_partials(part, n_blocks, out, gate=None):
    """out[k] = sum_b part[b, k] for b < n_blocks (deterministic order)."""
    dev = part.device
    cols = part.shape[1]
    if n_blocks > part.shape[0]:
        raise ValueError("n_blocks exceeds partial rows")
    lib().colsum_partials(_chk(part, torch.float64, "part", None, dev), int(n_blocks), int(cols),
                          _chk(out, torch.float64, "out", (cols,), dev), _gate_ptr(gate, dev), _stream())


def alpha_newton(scalars, num_docs, K, estimate, params, alpha_out):
    """Device lda-c opt_alpha: params[0:2] <- (alpha, lgamma(K alpha) - K lgamma(alpha))."""
    dev = params.device
    lib().alpha_newton(_chk(scalars, torch.float64, "scalars", (2,), dev), float(num_docs), int(K), bool(estimate),
                       _chk(params, torch.float64, "params", (PARAM_COUNT,), dev),
                       _chk(alpha_out, torch.float64, "alpha_out", (1,), dev), _stream())


def em_control(scalars, params, ctl, hist):
    """Device EM convergence test after one iteration (csrc/hip/em_control.hip)."""
    dev = params.device
    slots = hist.numel() // HIST_COLS
    lib().em_control(_chk(scalars, torch.float64, "scalars", (2,), dev),
                     _chk(params, torch.float64, "params", (PARAM_COUNT,), dev),
                     _chk(ctl, torch.float64, "ctl", (8,), dev),
                     _chk(hist, torch.float64, "hist", (slots * HIST_COLS,), dev),
                     int(slots), _stream())


def _bad(name):
    raise ValueError(f"{name}: buffer too small")


def score_events(theta, phi, K, dflt, doc_a, word_a, doc_b, word_b, tol):
    """Returns (score_a, score_b|None, key, flag) as new device tensors."""
    n = doc_a.numel()
    dev = doc_a.device
    D = theta.shape[0]
    V = phi.shape[0]
    if theta.dim() != 2 or phi.dim() != 2 or theta.shape[1] < K or phi.shape[1] < K:
        raise ValueError("theta/phi must be [*, >=K]")
    if theta.shape[1] != phi.shape[1]:
        raise ValueError("theta and phi row strides differ")
    Kr = theta.shape[1]
    if Kr != K:
        theta = theta[:, :K].contiguous()
        phi = phi[:, :K].contiguous()
    # index bounds (host check before a gather kernel touches memory)
    for name, idx, lim in (("doc_a", doc_a, D), ("word_a", word_a, V), ("doc_b", doc_b, D), ("word_b", word_b, V)):
        if idx is None:
            continue
        if idx.numel() != n:
            raise ValueError(f"{name}: length mismatch")
        if n and (int(idx.max()) >= lim or int(idx.min()) < -1):
            raise ValueError(f"{name}: index out of range")
    sa = torch.empty(n, dtype=torch.float64, device=dev)
    sb = torch.empty(n, dtype=torch.float64, device=dev) if doc_b is not None else None
    key = torch.empty(n, dtype=torch.float64, device=dev)
    flag = torch.empty(n, dtype=torch.uint8, device=dev)
    if n == 0:
        return sa, sb, key, flag
    lib().score_events(
        _chk(theta, torch.float64, "theta", (D, K), dev), _chk(phi, torch.float64, "phi", (V, K), dev),
        int(K), float(dflt),
        _chk(doc_a, torch.int32, "doc_a", (n,), dev), _chk(word_a, torch.int32, "word_a", (n,), dev),
        _chk(doc_b, torch.int32, "doc_b", (n,), dev) if doc_b is not None else 0,
        _chk(word_b, torch.int32, "word_b", (n,), dev) if word_b is not None else 0,
        int(n), float(tol), sa.data_ptr(), sb.data_ptr() if sb is not None else 0, key.data_ptr(),
        flag.data_ptr(), _stream(),
    )
    return sa, sb, key, flag


def flow_words(hour, minute, second, port_a, port_b, ipkt, ibyt, time_cuts, ibyt_cuts, ipkt_cuts):
    n = hour.numel()
    dev = hour.device
    cols = [hour, minute, second, port_a, port_b, ipkt, ibyt]
    names = ["hour", "minute", "second", "port_a", "port_b", "ipkt", "ibyt"]
    ptrs = [_chk(c, torch.float64, nm, (n,), dev) for c, nm in zip(cols, names)]
    cuts = [time_cuts, ibyt_cuts, ipkt_cuts]
    cptr = [_chk(c, torch.float64, "cuts", None, dev) for c in cuts]
    out = dict(
        time=torch.empty(n, dtype=torch.float64, device=dev),
        time_bin=torch.empty(n, dtype=torch.int8, device=dev),
        ibyt_bin=torch.empty(n, dtype=torch.int8, device=dev),
        ipkt_bin=torch.empty(n, dtype=torch.int8, device=dev),
        word_port=torch.empty(n, dtype=torch.float64, device=dev),
        p_case=torch.empty(n, dtype=torch.int8, device=dev),
        src_prefix=torch.empty(n, dtype=torch.int8, device=dev),
        dst_prefix=torch.empty(n, dtype=torch.int8, device=dev),
    )
    if n == 0:
        return out
    lib().flow_words(
        *ptrs, cptr[0], time_cuts.numel(), cptr[1], ibyt_cuts.numel(), cptr[2], ipkt_cuts.numel(), int(n),
        out["time"].data_ptr(), out["time_bin"].data_ptr(), out["ibyt_bin"].data_ptr(),
        out["ipkt_bin"].data_ptr(), out["word_port"].data_ptr(), out["p_case"].data_ptr(),
        out["src_prefix"].data_ptr(), out["dst_prefix"].data_ptr(), _stream(),
    )
    return out


def bin_columns(values, cuts):
    """bins[i, c] = #{cut in cuts[c] : values[c][i] > cut} (int8 [n, ncols])."""
    n = values[0].numel()
    dev = values[0].device
    vp = [_chk(v, torch.float64, "values", (n,), dev) for v in values]
    cp = [_chk(c, torch.float64, "cuts", None, dev) for c in cuts]
    out = torch.empty((n, len(values)), dtype=torch.int8, device=dev)
    if n == 0:
        return out
    lib().bin_columns(vp, cp, [int(c.numel()) for c in cuts], int(n), out.data_ptr(), _stream())
    return out


# ------------------------------------------------------- fp64 block Gauss-Seidel ---
# lda-c-faithful E-step (csrc/hip/lda_gs64.hip): double everywhere, gamma refreshed after every
# chunk of ceil(n / gs_updates) words (documents of <= gs_updates words: lda-c's per-word schedule).
GS_TINY, GS_TEAM1, GS_TEAM4, GS_TEAM8, GS_SMALL, GS_CHAIN = range(6)
GS_SMALL_MAX = 64   # csrc/hip/lda_gs64.hip kGsSmallMax


def gs_umax(KS: int = 0) -> int:
    """Largest U (gamma refreshes per sweep) of the fp64 engine: 4096 at every KS -- past 32 the chunk
    tables live in the c.phi rows (gs_team GMT, gs_chain; at KS > 32 also gs_smallw)."""
    return int(lib().gs_umax(int(KS)))


def gs_split_umax(KS: int) -> int:
    """Largest U of the split-document kernel: 4096 at KS > 32 (chunk tables past the LDS ones in a
    per-segment scratch, GSSplitPlan ``tab``), else its LDS tables' (64 at KS <= 52, else 32)."""
    return int(lib().gs_split_umax(int(KS)))


def gs_split_lds_umax(KS: int) -> int:
    """Largest U with the split kernel's chunk tables in LDS (64 at KS <= 52, else 32)."""
    return int(lib().gs_split_lds_umax(int(KS)))


def gs_tiny_max(KS: int) -> int:
    return int(lib().gs_tiny_max(int(KS)))


def _cphi_ptr(cphi, nnz, KS, dev, ent_base):
    """Device address of c.phi row 0 of the corpus: the whole [nnz, KS] buffer, or (``ent_base`` given)
    a window [rows, KS] holding corpus entries [ent_base, ent_base + rows) -- the kernels index rows by
    corpus entry, so the address is shifted back by ent_base rows.  The caller guarantees that every
    document of the launch has its entries inside the window (GSPlan(doc_range=...))."""
    if ent_base is None:
        return _chk(cphi, torch.float64, "cphi", (nnz, KS), dev)
    ptr = _chk(cphi, torch.float64, "cphi", None, dev)
    if cphi.dim() != 2 or cphi.shape[1] != KS or not (0 <= int(ent_base) and int(ent_base) + cphi.shape[0] <= nnz):
        raise ValueError(f"cphi window {tuple(cphi.shape)} at entry {ent_base} does not fit [{nnz}, {KS}]")
    return ptr - int(ent_base) * KS * 8


class GSStage:
    """Staged beta rows of one kGsTeam8 launch (KS <= 32): every document of ``order`` gets its rows
    copied in document order into one buffer, tiled [ceil(n / 64)][KS / 2][64] double2, refilled by
    ``gs_stage`` after each M-step.  The longest document's kernel then gathers 64 consecutive words
    as 16-byte-contiguous runs (one CU walks those rows U x 20 times per E-step) instead of 64
    scattered 8 KS-byte rows; the copy itself is spread over the whole GPU.  Costs n x KS x 8 bytes."""

    def __init__(self, order, doc_ptr_host, KS: int, device):
        import numpy as np
        if KS > 32 or KS % 2:
            raise ValueError("staged rows need an even KS <= 32")
        o = np.asarray(order.cpu().numpy() if torch.is_tensor(order) else order, np.int64)
        dp = np.asarray(doc_ptr_host, np.int64)
        per = (KS // 2) * 64
        off = np.zeros(o.size, np.int64)
        ents, cnts = [], []
        nt = 0
        for i, d in enumerate(o):
            if d < 0:
                continue
            s0, n = int(dp[d]), int(dp[d + 1] - dp[d])
            T = -(-n // 64)
            off[i] = nt * per
            ents.append(s0 + 64 * np.arange(T, dtype=np.int64))
            cnts.append(np.minimum(64, n - 64 * np.arange(T, dtype=np.int64)))
            nt += T
        self.KS, self.n_tiles = int(KS), nt
        cat = lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.int64)
        self.tile_ent = torch.from_numpy(cat(ents).astype(np.int32)).to(device)
        self.tile_cnt = torch.from_numpy(cat(cnts).astype(np.int32)).to(device)
        self.stage_off = torch.from_numpy(off).to(device)
        self.buf = torch.zeros(max(nt, 1) * per * 2, dtype=torch.float64, device=device)

    @property
    def nbytes(self) -> int:
        return self.n_tiles * (self.KS // 2) * 64 * 16


def gs_stage(beta, word_idx, st: "GSStage", gate=None):
    """Refill the staged rows of ``st`` from ``beta`` (after every M-step, before the team8 launch);
    ``gate``: the EM loop's done flag (a converged loop's queued iterations skip the copy)."""
    V, KS = beta.shape
    dev = beta.device
    if KS != st.KS:
        raise ValueError(f"staged rows of KS {st.KS}, beta has {KS}")
    if st.n_tiles == 0:
        return
    lib().gs_stage(_chk(beta, torch.float64, "beta", (V, KS), dev), _chk(word_idx, torch.int32, "word_idx", None, dev),
                   _chk(st.tile_ent, torch.int32, "tile_ent", (st.n_tiles,), dev),
                   _chk(st.tile_cnt, torch.int32, "tile_cnt", (st.n_tiles,), dev), st.n_tiles,
                   _chk(st.buf, torch.float64, "stage", None, dev), int(KS), _gate_ptr(gate, dev), _stream())


def _need_pad_row(t):
    """The E-step kernels load a row's topic lanes at constant offsets: lanes past KS read into the next
    row, the last row's into one pad row past the table (LDAEngine allocates beta as [V + 1, KS] and the
    c.phi rows as [nnz + 1, KS], and hands the kernels the views without it)."""
    V, KS = t.shape
    if t.untyped_storage().nbytes() < (t.storage_offset() + (V + 1) * KS) * t.element_size():
        raise ValueError("the table needs a pad row past its last row ([n + 1, KS] storage, view [:n])")


def gs_estep(doc_ptr, word_idx, counts, order, beta, K, gs_updates, params, gamma, cphi, lik, alpha_ss, iters, variant,
             dbg=None, ent_base=None, stage: Optional["GSStage"] = None):
    """One launch of the fp64 block Gauss-Seidel E-step over the documents in ``order``.
    ``params``: the device parameter block {alpha, lgamma constant, VAR_MAX_ITER, VAR_CONVERGED, done}.
    ``ent_base``: ``cphi`` is a window starting at that corpus entry (_cphi_ptr).
    ``stage``: the GSStage of this (kGsTeam8) launch, filled by ``gs_stage`` from the current beta."""
    D = doc_ptr.numel() - 1
    nnz = word_idx.numel()
    V, KS = beta.shape
    if KS not in compiled_ks():
        raise ValueError(f"beta row stride {KS} has no compiled kernel")
    if not (0 < K <= KS):
        raise ValueError("K out of range")
    if not (1 <= int(gs_updates) <= gs_umax(KS)):
        raise ValueError(f"gs_updates must be in [1, {gs_umax(KS)}] at KS {KS}")
    if variant not in (GS_TINY, GS_TEAM1, GS_TEAM4, GS_TEAM8, GS_SMALL, GS_CHAIN):
        raise ValueError(f"unknown gs variant {variant}")
    dev = beta.device
    args = [
        _chk(doc_ptr, torch.int32, "doc_ptr", (D + 1,), dev),
        _chk(word_idx, torch.int32, "word_idx", (nnz,), dev),
        _chk(counts, torch.float32, "counts", (nnz,), dev),
        _chk(order, torch.int32, "order", None, dev), order.numel(),
        _chk(beta, torch.float64, "beta", (V, KS), dev), int(K), int(KS), int(gs_updates),
        _params_ptr(params, dev) or _bad("params"),
        _chk(gamma, torch.float64, "gamma", (D, KS), dev),
        _cphi_ptr(cphi, nnz, KS, dev, ent_base),
        _chk(lik, torch.float64, "lik", (D,), dev),
        _chk(alpha_ss, torch.float64, "alpha_ss", (D,), dev),
        _chk(iters, torch.int32, "iters", (D,), dev),
        int(variant), _stream(), 0 if dbg is None else _chk(dbg, torch.int64, "dbg", (16,), dev),
        0 if stage is None else _chk(stage.buf, torch.float64, "stage", None, dev),
        0 if stage is None else _chk(stage.stage_off, torch.int64, "stage_off", (order.numel(),), dev),
    ]
    _need_pad_row(beta)
    if stage is not None and (variant != GS_TEAM8 or KS != stage.KS):
        raise ValueError("staged rows: kGsTeam8 launches of the stage's KS only")
    if order.numel() == 0:
        return
    lib().gs_estep(*args)


def gs_suff64(word_ptr, csc_ent, plan: "SuffPlan", cphi, cw, part, gate=None, scalars=None, base=None):
    """class_word[w] = sum of the cphi rows of w's corpus entries (CSC order, fp64, no atomics) + per-workgroup
    partial rows part[b] = {lik slice, alpha_ss slice, column sums} for ``colsum_partials``.
    ``base`` [V, KS] (optional): added to each written row first (cw[w] = base[w] + sum)."""
    V, KS = cw.shape
    nnz = cphi.shape[0]            # csc_ent may be a subset of the corpus entries (csc_subset)
    dev = cw.device
    if plan.covers_all and plan.order.numel() != V:
        raise ValueError("suff plan does not cover the vocabulary")
    if plan.order.numel() == 0:
        return
    if csc_ent.numel() > nnz:
        raise ValueError("csc_ent longer than the corpus")
    if part.dim() != 2 or part.shape[1] != KS + 2 or part.shape[0] < max(plan.n_blocks, 1):
        raise ValueError(f"part: shape {tuple(part.shape)}, expected [>= {plan.n_blocks}, {KS + 2}]")
    if KS > 32:
        _need_pad_row(cphi)        # paired row loads read up to one row past the last entry
    if scalars is None:
        lik = ass = 0
        lo = hi = 0
    else:
        D = scalars[0].numel()
        lik, ass, lo, hi = _scalar_slice(scalars, D, dev)
    lib().gs_suff64(
        _chk(word_ptr, torch.int32, "word_ptr", (V + 1,), dev), _chk(csc_ent, torch.int32, "csc_ent", None, dev),
        _chk(plan.order, torch.int32, "order", (plan.order.numel(),), dev), plan.n_heavy, plan.n_medium, plan.n_light,
        _chk(cphi, torch.float64, "cphi", (nnz, KS), dev), _chk(cw, torch.float64, "cw", (V, KS), dev),
        _chk(part, torch.float64, "part", None, dev), lik, ass, lo, hi, int(KS), _gate_ptr(gate, dev), _stream(),
        0 if base is None else _chk(base, torch.float64, "base", (V, KS), dev))


def csc_subset(word_ptr, csc_ent, csc_doc, doc_mask):
    """(word_ptr, csc_ent) of the CSC slots whose document is in ``doc_mask`` (bool [D], device), slot
    order kept; plus the per-word entry counts on the host (for a SuffPlan)."""
    from . import sortgroup as SG
    keep = SG.gather(doc_mask, csc_doc)
    ce, before = SG.compact(csc_ent, keep)       # before[s]: kept slots ahead of slot s
    ptr = SG.gather(before, word_ptr)            # word w's kept slots start where its slots do
    return ptr.to(torch.int32), ce.contiguous(), (ptr[1:] - ptr[:-1]).cpu().numpy()


def suff_group_plan(lens, V: int):
    """Host plan of the per-stream suff-stats (LDAEngine._build_suff_groups).  lens[g]: entries of each word
    in stream g's documents.  Per stream: ``unique`` -- words whose entries all lie in g (stream 0 also
    takes the words with no entry, written as zero rows), ``multi`` -- words shared with another stream,
    whose rows go to scratch rows off[g] + i; the combine CSC (wp, ce) lists, per shared word, its scratch
    rows in stream order.  None when no word is shared."""
    import numpy as np
    present = np.stack([np.asarray(ln) > 0 for ln in lens])
    nper = present.sum(0)
    multi = nper > 1
    unique, mlist, off = [], [], []
    rows = 0
    wcat, gcat, rcat = [], [], []
    for gi in range(len(lens)):
        u = np.flatnonzero(present[gi] & ~multi)
        if gi == 0:
            u = np.union1d(u, np.flatnonzero(nper == 0))
        mw = np.flatnonzero(present[gi] & multi)
        unique.append(u), mlist.append(mw), off.append(rows)
        if mw.size:
            wcat.append(mw), gcat.append(np.full(mw.size, gi)), rcat.append(rows + np.arange(mw.size))
            rows += int(mw.size)
    if rows == 0:
        return None
    w_all, g_all, r_all = np.concatenate(wcat), np.concatenate(gcat), np.concatenate(rcat)
    o = np.lexsort((g_all, w_all))                   # by word, then stream order
    cnt = np.bincount(w_all, minlength=V).astype(np.int64)
    wp = np.zeros(V + 1, np.int64)
    wp[1:] = np.cumsum(cnt)
    return dict(unique=unique, multi=mlist, off=off, rows=rows, wp=wp, ce=r_all[o], cnt=cnt,
                shared=np.flatnonzero(multi))


def csc_compact(word_ptr, csc_ent, words):
    """(word_ptr, csc_ent) of the CSC columns ``words`` (host ids), renumbered 0 .. len(words) - 1, slot
    order kept (a compact sub-CSC for a gs_suff64 pass into a scratch of len(words) rows)."""
    import numpy as np
    from . import sortgroup as SG
    dev = word_ptr.device
    w = torch.from_numpy(np.asarray(words, np.int64)).to(dev)
    st = SG.gather(word_ptr, w).long()
    ln = SG.gather(word_ptr, w + 1).long() - st
    ptr = torch.zeros(w.numel() + 1, dtype=torch.int64, device=dev)
    ptr[1:] = torch.cumsum(ln, 0)
    tot = int(ptr[-1])
    idx = SG.gather(st - ptr[:-1], SG.segment_ids(ln, tot)) + torch.arange(tot, device=dev)
    return ptr.to(torch.int32), SG.gather(csc_ent, idx).contiguous()


def gs_mstep_control(cw, class_total, beta, K, scalars, params, ctl, hist, done_count, rows=None, newton=None,
                     stages=(), word_idx=None):
    """fp64 M-step (beta = cw / class_total, exp(-100) floor) + alpha Newton + device EM control step.
    ``stages`` (at most 2 GSStage, with the corpus ``word_idx``): their staged rows refilled by trailing
    workgroups of the same launch, from cw / class_total (bit-equal to gs_stage from the new beta)."""
    V, KS = cw.shape
    dev = cw.device
    sets = []
    for st in stages:
        if st.KS != KS:
            raise ValueError(f"staged rows of KS {st.KS}, cw has {KS}")
        if st.n_tiles:
            sets.append((_chk(st.tile_ent, torch.int32, "tile_ent", (st.n_tiles,), dev),
                         _chk(st.tile_cnt, torch.int32, "tile_cnt", (st.n_tiles,), dev),
                         _chk(st.buf, torch.float64, "stage", None, dev), int(st.n_tiles)))
    if len(sets) > 2:
        raise ValueError("gs_mstep_control: at most 2 staged sets")
    wi = _chk(word_idx, torch.int32, "word_idx", None, dev) if sets else 0
    slots = hist.numel() // HIST_COLS
    n_rows = 0 if rows is None else int(rows.numel())
    rows_ptr = 0 if rows is None else _chk(rows, torch.int32, "rows", (n_rows,), dev)
    lib().gs_mstep_control(
        _chk(cw, torch.float64, "cw", (V, KS), dev), _chk(class_total, torch.float64, "class_total", (KS,), dev),
        _chk(beta, torch.float64, "beta", (V, KS), dev), int(V), int(K), int(KS),
        _chk(scalars, torch.float64, "scalars", (2,), dev), _chk(params, torch.float64, "params", (PARAM_COUNT,), dev),
        _chk(ctl, torch.float64, "ctl", (8,), dev), _chk(hist, torch.float64, "hist", (slots * HIST_COLS,), dev),
        int(slots), _chk(done_count, torch.int32, "done_count", (1,), dev), _stream(), rows_ptr, n_rows,
        0 if newton is None else 1, 0 if newton is None else int(bool(newton[0])),
        0.0 if newton is None else float(newton[1]),
        0 if newton is None else _chk(newton[2], torch.float64, "alpha_out", (1,), dev), wi, sets)


def gs_mstep(cw, class_total, beta, K, gate=None):
    V, KS = cw.shape
    dev = cw.device
    lib().gs_mstep(_chk(cw, torch.float64, "cw", (V, KS), dev),
                   _chk(class_total, torch.float64, "class_total", (KS,), dev),
                   _chk(beta, torch.float64, "beta", (V, KS), dev), int(V), int(K), int(KS), _gate_ptr(gate, dev),
                   _stream())


def split_spec(KS: int) -> dict:
    """The split-document plan of ONI_GS_SPLIT_MIN = 'N[,g=G][,batches=B][,words=W]': documents longer
    than N words split (default 2048 at KS > 32, 0 = off at KS <= 32), at most G workgroups per document
    (SPLIT_MAX_SEG), B launch batches (1), W words of a chunk per workgroup (0: the split kernel's
    prefetched rounds, split_seg_words)."""
    from .. import knobs
    spec = (knobs.get("ONI_GS_SPLIT_MIN") or "").strip()
    out = dict(min=2048 if KS > 32 else 0, g=SPLIT_MAX_SEG, batches=1, words=0)
    if spec:
        head, *rest = [x.strip() for x in spec.split(",")]
        if head:
            out["min"] = int(head)
        for kv in rest:
            k, v = kv.split("=")
            if k.strip() not in ("g", "batches", "words"):
                raise ValueError(f"ONI_GS_SPLIT_MIN: unknown field {k!r} in {spec!r}")
            out[k.strip()] = int(v)
    return out


def gs_split_launch_cap(KS: int) -> int:
    """Workgroups per gs_split launch: 3/4 of the co-resident capacity (occupancy API x CUs), so a
    launch's segments are resident together with room for the other streams' buckets;
    ONI_SPLIT_MAX_BLOCKS lowers it (tests, shared / partitioned GPUs)."""
    from .. import knobs
    cap = max(1, int(lib().gs_split_capacity(int(KS))) * 3 // 4)
    env = knobs.get("ONI_SPLIT_MAX_BLOCKS")
    if env:
        cap = max(1, min(cap, int(env)))
    return cap


SPLIT_MAX_SEG = 128        # csrc/hip/lda_gs64.hip kSplitMaxSeg2 (segments per document)
SPLIT_MAX_SEG_GATHER = 16  # kSplitMaxSeg: up to here one batched gather per chunk, above it the two-phase exchange


def gs_team8_words(KS: int) -> int:
    """Words of a chunk one 8-wave fp64 workgroup holds in its prefetched rounds (TeamShape<KS, 8>:
    slots x RMAX)."""
    tg = 4 if KS <= 32 else (8 if KS <= 64 else 16)
    kpl = -(-KS // tg)
    return 8 * (64 // tg) * (8 if kpl <= 5 else 4)


def split_seg_words(KS: int) -> int:
    """Words of a chunk one split segment holds in its prefetched rounds: the split kernel's 7 word waves
    (gs_splitw: TeamShape<KS, 8> slots and RMAX) -- a segment past it streams the rest one gather latency
    per round."""
    return gs_team8_words(KS) * 7 // 8


def split_seg_target(KS: int) -> int:
    """Smallest useful share of a chunk per split segment (words), the water-filling's cap on a document's
    segments (G <= ceil(W / target)): the split kernel's prefetched rounds at K = 100 (112 words); at KS <= 64
    (8-lane topic groups, 224 prefetched words) 96 -- the 1-day corpus at K = 50 per EM iteration: 3.15 ms with
    the prefetch-sized cap (its longest document on 4 segments), 2.94 / 2.58 / 2.88 / 3.6 ms with fixed
    shares of 128 / 96 / 64 / 48 words (profiles/r6z_split_k50.md)."""
    return 96 if KS <= 64 else split_seg_words(KS)


def split_chain_cycles(n: int, U: int, G: int, KS: int) -> float:
    """Modelled cycles of one chunk of an n-word document on G segments (G = 1: the 8-wave team kernel),
    for the plan's segment allocation only (profiles/r6_split.md): a word-phase term per word of the
    segment's share plus the exchange (one batched gather up to 16 segments, two round trips beyond)."""
    W = -(-n // U)
    per = -(-W // G)
    sw = split_seg_words(KS)
    # prefetched rounds cost ~issue + compute; streamed rounds a gather latency each
    word = 40.0 * min(per, sw) + (1800.0 * -(-(per - sw) // sw) if per > sw else 0.0) + 2000.0
    if G == 1:
        return word
    # the exchange's steps past 4 segments grow with the granules a segment reads: (KS + 1) columns each.
    # Fitted at K = 100; at K = 50 the unscaled steps stopped the 1-day corpus' longest document at 4 segments,
    # 3.15 ms per EM iteration against 2.58 with 8 (profiles/r6z_split_k50.md)
    step = 0.0 if G <= 4 else 2500.0 if G <= 8 else 8000.0 if G <= SPLIT_MAX_SEG_GATHER else 6000.0
    xch = 4000.0 + step * (KS + 1) / 101.0
    return word + xch + 1500.0


class GSSplitPlan:
    """Launch batches of the fp64 split-document kernel (gs_split): document d of n words (W = ceil(n / U)
    words per chunk) gets G workgroups, each taking 1/G of every chunk; a batch holds
    <= gs_split_launch_cap(KS) workgroups (co-resident, so the per-chunk exchange cannot deadlock).

    G per document is water-filled over the launch cap: every candidate starts at G = 1 (the 8-wave team
    kernel), and the document whose modelled chunk time (split_chain_cycles) is the largest gets more
    segments, until the cap is spent or that document is at its most useful G = ceil(W / seg_words) (at most
    SPLIT_MAX_SEG): the launch shortens the longest chain first; the budget left gives the other candidates
    two segments each, longest first.  Documents still at G = 1 stay with the team kernel (``leftover``),
    unless ``max_batches`` > 1 (ONI_GS_SPLIT_MIN batches=B, default 1) allows more batches of the rest
    (back to back on one stream: a later batch lengthens the critical path)."""

    def __init__(self, doc_ids, lengths, KS: int, gs_updates: int, device, seg_words: int = 0,
                 max_seg: int = 0, max_batches: int = 0):
        import heapq
        import numpy as np
        self.KS = int(KS)
        self.max_blocks = gs_split_launch_cap(KS)
        sp = split_spec(KS)
        # an explicit segment size (ONI_GS_SPLIT_MIN words=W, or the argument) fixes G = clamp(ceil(W / words),
        # 2, max_seg) per document, longest first; otherwise the modelled water-filling (_allocate)
        # KS <= 64: fixed 96-word shares by default -- measured ahead of the water-filling there (2.58 vs 2.74 ms
        # per EM iteration at K = 50, profiles/r6z_split_k50.md), where the model was fitted at K = 100
        self.fixed = bool(int(seg_words) or sp["words"]) or self.KS <= 64
        self.seg_words = int(seg_words) or sp["words"] or split_seg_target(KS)
        # KS <= 32: the single-round gather only (gs_splitw has no two-phase exchange in the narrow layout)
        max_seg = min(int(max_seg) or sp["g"], self.max_blocks,
                      SPLIT_MAX_SEG if self.KS > 32 else SPLIT_MAX_SEG_GATHER)
        max_batches = int(max_batches) or sp["batches"]
        U = int(gs_updates)
        self.U = U
        self.tab_lds = U <= gs_split_lds_umax(self.KS)
        self.segments = {}
        self.batches = []
        self.leftover = []
        todo = [int(d) for d in doc_ids]
        while todo and len(self.batches) < max_batches:
            G = self._allocate(todo, lengths, U, max_seg)
            docs = [(d, G[d]) for d in todo if G[d] >= 2]
            if not docs:
                break
            for d, g in docs:
                self.segments[d] = g
            self.batches.append(self._make(docs, lengths, device))
            done = {d for d, _ in docs}
            todo = [d for d in todo if d not in done]
        self.leftover = todo
        self.n_docs = len(self.segments)

    def _allocate(self, docs, lengths, U, max_seg):
        """Water-filling: segments to the document with the longest modelled chunk, within the cap."""
        import heapq
        G = {d: 1 for d in docs}
        if self.fixed:
            used = 0
            for d in docs:
                W = -(-int(lengths[d]) // U)
                g = min(max(2, -(-W // self.seg_words)), max_seg, W)
                if g >= 2 and used + g <= self.max_blocks:
                    G[d] = g
                    used += g
            return G
        gmax = {}
        for d in docs:
            W = -(-int(lengths[d]) // U)
            # a document with W >= 2 words per chunk can always take two segments
            gmax[d] = 1 if W < 2 else max(2, min(max_seg, W, -(-W // self.seg_words)))
        t = lambda d, g: split_chain_cycles(int(lengths[d]), U, g, self.KS)   # noqa: E731
        heap = [(-t(d, 1), d) for d in docs if gmax[d] >= 2]
        heapq.heapify(heap)
        used = 0
        while heap:
            tc, d = heapq.heappop(heap)
            g = G[d]
            # the fewest more segments that shorten it (the exchange's cost steps up at 5, 9 and 17 segments);
            # one workgroup -> G segments costs G launch slots
            gn = next((x for x in range(max(2, g + 1), gmax[d] + 1)
                       if used + x - (g if g > 1 else 0) <= self.max_blocks and t(d, x) < -tc), None)
            if gn is None:
                break     # the longest chain cannot shorten further: the rest cannot set the launch time
            used += gn - (g if g > 1 else 0)
            G[d] = gn
            heapq.heappush(heap, (-t(d, gn), d))
        # the budget left: two segments for each remaining candidate, longest first -- a co-resident split
        # launch is dispatched ahead of the short-document floods, where a 512-thread team workgroup can
        # queue behind them (K = 50: 4.5 -> 3.4 ms per EM iteration, profiles/r3_tuning_log.md)
        for d in docs:
            if G[d] == 1 and gmax[d] >= 2 and used + 2 <= self.max_blocks:
                G[d] = 2
                used += 2
        return G

    def _make(self, docs, lengths, device):
        import numpy as np
        sd, si, sc, sb, slot = [], [], [], [], []
        for j, (d, G) in enumerate(docs):
            base = len(sd)
            for q in range(G):
                sd.append(d), si.append(q), sc.append(G), sb.append(base), slot.append(j)
        t = lambda a: torch.tensor(np.asarray(a, np.int32), device=device)
        nb = len(sd)
        gmx = SPLIT_MAX_SEG if self.KS > 32 else SPLIT_MAX_SEG_GATHER
        if sc and max(sc) > gmx:
            raise ValueError(f"gs_split: {max(sc)} segments per document > {gmx} at KS {self.KS}")
        if nb > self.max_blocks:
            raise ValueError(f"gs_split: {nb} workgroups > the launch cap {self.max_blocks}")
        # U past the LDS chunk tables: per-segment tables in a scratch ([n_blocks][tab_rows][2][KS] doubles),
        # tab_rows = the batch's largest chunk count (<= U)
        tab_rows = 0 if self.tab_lds else max(-(-int(lengths[d]) // -(-int(lengths[d]) // self.U)) for d, _ in docs)
        gr = 2 * (self.KS + 1)
        return dict(seg_doc=t(sd), seg_index=t(si), seg_count=t(sc), seg_base=t(sb), doc_slot=t(slot), n_blocks=nb,
                    # tagged granules {uint32 half of a double, uint32 tag}: [2][n_blocks][2 (KS + 1)] partials,
                    # then [2][docs][2 (KS + 1)] totals (the two-phase exchange past 16 segments)
                    xchg=torch.zeros(2 * nb * gr + 2 * len(docs) * gr, dtype=torch.int64, device=device),
                    counter=torch.zeros(2 * len(docs), dtype=torch.int32, device=device),
                    error=torch.zeros(1, dtype=torch.int32, device=device), docs=len(docs), tab_rows=tab_rows,
                    tab=(torch.empty(nb * tab_rows * 2 * self.KS, dtype=torch.float64, device=device)
                         if tab_rows else None))

    def chunk_sums(self, doc_ptr, counts) -> None:
        """Each batch document's chunk count sums ([docs][max nch] doubles, exact: integer counts) from the
        corpus' host doc_ptr / counts, for the kernel's C_j initialisation (built once per plan)."""
        import numpy as np
        for b in self.batches:
            docs = b["seg_doc"].cpu().numpy()[b["seg_base"].cpu().numpy() == np.arange(b["n_blocks"])]
            rows = []
            for d in docs:
                s0, s1 = int(doc_ptr[d]), int(doc_ptr[d + 1])
                n = s1 - s0
                W = -(-n // self.U)
                c = np.asarray(counts[s0:s1], np.float64)
                nch = -(-n // W)
                rows.append(np.add.reduceat(c, np.arange(0, n, W)) if n else np.zeros(0))
                assert rows[-1].size == nch
            width = max(1, max(r.size for r in rows))
            cs = np.zeros((len(rows), width), np.float64)
            for i, r in enumerate(rows):
                cs[i, :r.size] = r
            b["csum"] = torch.from_numpy(cs).to(b["seg_doc"].device)
            b["csum_u"] = self.U

    def scratch_bytes(self) -> int:
        """Device bytes of the batches' chunk-table scratch (counted in the c.phi budget)."""
        return sum(b["tab"].numel() * 8 for b in self.batches if b.get("tab") is not None)


def gs_split(doc_ptr, word_idx, counts, beta, K, gs_updates, params, gamma, cphi, lik, alpha_ss, iters, batch,
             dbg=None, ent_base=None):
    """One launch of the fp64 split-document E-step over one GSSplitPlan batch.  dbg: optional int64[8]
    phase timer of workgroup 0 (word phase, barrier 1, publish + gather, barrier 2, refresh, barrier 3,
    sweep end, chunks)."""
    D = doc_ptr.numel() - 1
    nnz = word_idx.numel()
    V, KS = beta.shape
    dev = beta.device
    nb = batch["n_blocks"]
    if KS not in compiled_ks():
        raise ValueError(f"beta row stride {KS} has no compiled kernel")
    if not (0 < K <= KS) or not (1 <= int(gs_updates) <= gs_split_umax(KS)):
        raise ValueError("K or gs_updates out of range")
    for k in ("seg_doc", "seg_index", "seg_count", "seg_base", "doc_slot"):
        _chk(batch[k], torch.int32, k, (nb,), dev)
    _need_pad_row(beta)
    lib().gs_split(
        _chk(doc_ptr, torch.int32, "doc_ptr", (D + 1,), dev), _chk(word_idx, torch.int32, "word_idx", (nnz,), dev),
        _chk(counts, torch.float32, "counts", (nnz,), dev), _chk(beta, torch.float64, "beta", (V, KS), dev),
        int(K), int(KS), int(gs_updates), _params_ptr(params, dev) or _bad("params"),
        _chk(gamma, torch.float64, "gamma", (D, KS), dev), _cphi_ptr(cphi, nnz, KS, dev, ent_base),
        _chk(lik, torch.float64, "lik", (D,), dev), _chk(alpha_ss, torch.float64, "alpha_ss", (D,), dev),
        _chk(iters, torch.int32, "iters", (D,), dev),
        batch["seg_doc"].data_ptr(), batch["seg_index"].data_ptr(), batch["seg_count"].data_ptr(),
        batch["seg_base"].data_ptr(), batch["doc_slot"].data_ptr(), int(nb),
        _chk(batch["xchg"], torch.int64, "xchg", (2 * (nb + batch["docs"]) * 2 * (KS + 1),), dev),
        _chk(batch["counter"], torch.int32, "counter", (2 * batch["docs"],), dev), int(batch["docs"]),
        _chk(batch["error"], torch.int32, "error", (1,), dev), _stream(),
        0 if dbg is None else _chk(dbg, torch.int64, "dbg", (8,), dev),
        *_split_tab(batch, nb, int(gs_updates), KS, dev, doc_ptr), *_split_csum(batch, int(gs_updates), dev))


def _split_csum(batch, U, dev):
    """(address, stride) of the batch's chunk count sums (GSSplitPlan.chunk_sums), (0, 0) if not built."""
    cs = batch.get("csum")
    if cs is None:
        return 0, 0
    if batch.get("csum_u") != U:
        raise ValueError(f"gs_split: chunk sums built for U = {batch.get('csum_u')}, launched with U = {U}")
    _chk(cs, torch.float64, "csum", (batch["docs"], cs.shape[1]), dev)
    return cs.data_ptr(), int(cs.shape[1])


def _split_tab(batch, nb, U, KS, dev, doc_ptr):
    """(scratch address, rows per workgroup) of the split batch's chunk tables (required past the LDS
    tables' U); the rows must cover every document's chunk count (the kernel also checks)."""
    tab = batch.get("tab")
    if U > gs_split_lds_umax(KS):
        rows = int(batch.get("tab_rows") or 0)
        if tab is None or rows <= 0 or tab.numel() < nb * rows * 2 * KS:
            raise ValueError(f"gs_split: U = {U} needs a chunk-table scratch of {nb} x rows x 2 x {KS} doubles")
        return _chk(tab, torch.float64, "tab", None, dev), rows
    return 0, 0


def gs_xsplit_rows(KS: int) -> int:
    """LDS row capacity of one gs_xsplit member (its words over every chunk of a sweep), 0: no kernel."""
    return int(exp_lib().gs_xsplit_rows(int(KS)))


class GSXSplitPlan:
    """Documents split over the CUs of one XCD each (gs_xsplit, csrc/hip/experimental/lda_xsplit.hip, even KS <= 32;
    measured not faster than one workgroup: profiles/r5_xcd_split.md).

    The first ``limit`` documents of ``doc_ids`` (longest first) that fit are taken.  Document d of n words
    (W = ceil(n / U) words per chunk) gets G one-wave members, each holding its
    ceil(W / G) words of every chunk in LDS: G >= the LDS minimum, ``members`` or as
    many as that takes, at most 32 (the CUs of an XCD).  Documents are first-fit packed into the 8 XCD
    groups (members of group x are blocks x, x + 8, ... of a grid of 8 x max-members blocks: one XCD
    under the observed round-robin dispatch); a document that fits no group stays with the team
    kernels (``leftover``).  Duck-types GSSplitPlan for the engine (segments, batches, n_docs)."""

    def __init__(self, doc_ids, lengths, KS: int, gs_updates: int, device, members: int = 0, groups: int = 8,
                 proto: int = 1, limit: int = 0):
        import numpy as np
        self.KS, U = int(KS), int(gs_updates)
        cap = gs_xsplit_rows(KS)
        if cap <= 0 or not 1 <= U <= 32:
            raise ValueError(f"gs_xsplit: no kernel for KS {KS} / U {U}")
        members = int(members)
        self.proto = int(proto)
        used = [0] * 8
        slots = [[] for _ in range(8)]          # per group: (doc, G)
        self.segments, self.leftover = {}, []
        for d in doc_ids:
            if limit and len(self.segments) >= limit:
                break
            n = int(lengths[d])
            W = -(-n // U)
            nch = -(-n // W)
            per = cap // nch                     # words of one chunk a member can hold
            gmin = -(-W // per) if per > 0 else 10 ** 9
            G = max(gmin, min(members, W) if members else gmin, 2)
            x = next((x for x in range(min(groups, 8)) if used[x] + G <= 32), None)
            if G > 32 or x is None or W < 2:
                self.leftover.append(int(d))
                continue
            slots[x].append((int(d), G))
            used[x] += G
            self.segments[int(d)] = G
        self.n_docs = len(self.segments)
        gmax = max(used) if self.n_docs else 0
        nb = 8 * gmax
        seg_doc = np.full(nb, -1, np.int32)
        seg_index = np.zeros(nb, np.int32)
        seg_count = np.ones(nb, np.int32)
        seg_base = np.zeros(nb, np.int32)
        doc_slot = np.zeros(nb, np.int32)
        row, slot = 0, 0
        for x in range(8):
            m = 0
            for d, G in slots[x]:
                for gi in range(G):
                    b = x + 8 * (m + gi)
                    seg_doc[b], seg_index[b], seg_count[b], seg_base[b], doc_slot[b] = d, gi, G, row, slot
                m += G
                row += G
                slot += 1
        t = lambda a: torch.from_numpy(a).to(device)
        self.batches = [] if not self.n_docs else [dict(
            x=True, seg_doc=t(seg_doc), seg_index=t(seg_index), seg_count=t(seg_count), seg_base=t(seg_base),
            doc_slot=t(doc_slot), n_blocks=nb, n_rows=row,
            # granules {lo, tag, hi, tag} (uint32): [2][n_rows][KS + 1][4]
            xchg=torch.zeros(2 * row * (self.KS + 1) * 4, dtype=torch.int32, device=device),
            counter=torch.zeros(2 * slot, dtype=torch.int32, device=device),
            error=torch.zeros(1, dtype=torch.int32, device=device),
            placed=torch.zeros(max(slot, 1), dtype=torch.int32, device=device), docs=slot, proto=self.proto)]


def gs_xsplit(doc_ptr, word_idx, counts, beta, K, gs_updates, params, gamma, cphi, lik, alpha_ss, iters, batch,
              dbg=None, ent_base=None):
    """One launch of the XCD-split E-step over a GSXSplitPlan batch.  dbg: optional int64[8] phase timer
    of member 0 of the first document (word phase + reduction, publish -> gathered, refresh, chunks)."""
    D = doc_ptr.numel() - 1
    nnz = word_idx.numel()
    V, KS = beta.shape
    dev = beta.device
    nb = batch["n_blocks"]
    if gs_xsplit_rows(KS) <= 0 or not (0 < K <= KS) or not (1 <= int(gs_updates) <= 32):
        raise ValueError("gs_xsplit: KS, K or gs_updates out of range")
    for k in ("seg_doc", "seg_index", "seg_count", "seg_base", "doc_slot"):
        _chk(batch[k], torch.int32, k, (nb,), dev)
    exp_lib().gs_xsplit(
        _chk(doc_ptr, torch.int32, "doc_ptr", (D + 1,), dev), _chk(word_idx, torch.int32, "word_idx", (nnz,), dev),
        _chk(counts, torch.float32, "counts", (nnz,), dev), _chk(beta, torch.float64, "beta", (V, KS), dev),
        int(K), int(KS), int(gs_updates), _params_ptr(params, dev) or _bad("params"),
        _chk(gamma, torch.float64, "gamma", (D, KS), dev), _cphi_ptr(cphi, nnz, KS, dev, ent_base),
        _chk(lik, torch.float64, "lik", (D,), dev), _chk(alpha_ss, torch.float64, "alpha_ss", (D,), dev),
        _chk(iters, torch.int32, "iters", (D,), dev),
        batch["seg_doc"].data_ptr(), batch["seg_index"].data_ptr(), batch["seg_count"].data_ptr(),
        batch["seg_base"].data_ptr(), batch["doc_slot"].data_ptr(), int(nb), int(batch["n_rows"]),
        _chk(batch["xchg"], torch.int32, "xchg", (2 * batch["n_rows"] * (KS + 1) * 4,), dev),
        _chk(batch["counter"], torch.int32, "counter", (2 * batch["docs"],), dev), int(batch["docs"]),
        _chk(batch["error"], torch.int32, "error", (1,), dev), int(batch["proto"]),
        _chk(batch["placed"], torch.int32, "placed", None, dev), _stream(),
        0 if dbg is None else _chk(dbg, torch.int64, "dbg", (8,), dev))


class GSPlan:
    """Length buckets of the fp64 block Gauss-Seidel E-step: (variant, int32 doc order) per launch.

    tiny (TG lanes per document, literal schedule) for n <= min(gs_tiny_max(KS), U); up to 256 words
    one wave per document at KS <= 32, 16 lanes per document at KS > 32 (gs_smallw); a 4-wave workgroup
    up to 2048; an 8-wave workgroup beyond."""
    EDGES = ((GS_TEAM8, 2048, None), (GS_TEAM4, 256, 2048), (GS_SMALL, None, 256))
    # KS <= 32: documents up to GS_SMALL_MAX words go to the 16-lanes-per-document kernel
    EDGES_NARROW = ((GS_TEAM8, 2048, None), (GS_TEAM4, 256, 2048), (GS_TEAM1, GS_SMALL_MAX, 256),
                    (GS_SMALL, None, GS_SMALL_MAX))

    def __init__(self, lengths, KS: int, gs_updates: int, device, split_min: Optional[int] = None,
                 doc_range=None, xsplit: Optional[dict] = None):
        import numpy as np
        self.KS = int(KS)
        L = np.asarray(lengths, dtype=np.int64)
        # doc_range (d0, d1): only documents d0 <= d < d1 (one c.phi window of the engine); the stable
        # sort of the range equals the range's documents in the stable sort of all of them
        self.doc_range = None if doc_range is None else (int(doc_range[0]), int(doc_range[1]))
        if self.doc_range is None:
            order = argsort_desc_stable(L).astype(np.int32)
        else:
            d0, d1 = self.doc_range
            order = (d0 + argsort_desc_stable(L[d0:d1])).astype(np.int32)
        # documents longer than split_min words: one document over several workgroups (gs_split);
        # default on for KS > 32 (the topic-group team kernels' chunk of a long document is bound
        # by one CU's row gathers), ONI_GS_SPLIT_MIN overrides (0: off; split_spec)
        # K > 32: 2048 (the whole team8 range) -- at 4096 the 2-4 k-word documents' 512-thread
        # workgroups were dispatched behind the short-document floods in some iterations (a bimodal
        # 2.75 / 4.5 ms team8 bucket); one co-resident split launch holds them all: K = 50 4.53 / 4.73
        # -> 3.36 / 3.34 ms per EM iteration (profiles/r3_tuning_log.md)
        if split_min is None:
            split_min = split_spec(KS)["min"]
        if int(gs_updates) > gs_split_umax(KS):
            split_min = 0       # KS <= 32: the split kernel's chunk tables live in LDS (U <= 32)
        self.split = None
        # xsplit = {docs: N, members: G, proto: P} (even KS <= 32): the N longest documents over the CUs of
        # one XCD each (gs_xsplit; an experiment, off by default: profiles/r5_xcd_split.md)
        xs = dict(xsplit or {})
        nx = int(xs.pop("docs", 0)) if KS <= 32 and KS % 2 == 0 and int(gs_updates) <= 32 else 0
        if nx > 0 and L.size and gs_xsplit_rows(KS) > 0:
            head = order[:nx + 16]
            head = head[L[head] > 2 * int(gs_updates)]
            xp = GSXSplitPlan(head, L, KS, gs_updates, device, limit=nx, **xs) if head.size else None
            if xp is not None and xp.n_docs:
                self.split = xp
                order = order[~np.isin(order, np.asarray(sorted(xp.segments), np.int64))]
                split_min = 0
        if split_min > 0 and (L > split_min).any():
            m = L[order] > split_min
            sp = GSSplitPlan(order[m], L, KS, gs_updates, device)
            if sp.n_docs:
                self.split = sp
                keep = np.ones(len(order), bool)
                keep[np.flatnonzero(m)] = ~np.isin(order[m], np.asarray(sorted(sp.segments), np.int64))
                order = order[keep]
        Ls = L[order]
        tiny = min(gs_tiny_max(KS), int(gs_updates))
        self.plan = []
        # team8 at KS <= 32: the longest document first in a workgroup order that gives it an XCD of its own
        # under round-robin dispatch (isolate_longest, a speed hint)
        iso = 1 if KS <= 32 else 0
        edges = self.EDGES_NARROW if KS <= 32 else self.EDGES
        if int(gs_updates) > 32:
            edges = self.wide_u_edges(int(gs_updates)) if KS > 32 else self.narrow_wide_u_edges(int(gs_updates))
        for var, lo, hi in edges:
            lo_ = tiny if lo is None else lo
            m = (Ls > lo_) if hi is None else ((Ls > lo_) & (Ls <= hi))
            if not m.any():
                continue
            o = order[m].copy()
            if var == GS_TEAM8 and iso > 0:
                o = self.isolate_longest(o, min(iso, 8))
            self.plan.append((var, torch.from_numpy(o).to(device)))
        m = Ls <= tiny
        if m.any():
            self.plan.append((GS_TINY, torch.from_numpy(order[m].copy()).to(device)))
        self.tiny_max = tiny
        # (the other buckets leaving the longest document's XCD to it measured slower twice and is gone:
        # 2.20 / 2.27 vs 2.18 / 2.18 ms, then 1.746 / 1.742 / 1.761 vs 1.734 / 1.733 / 1.739 ms per EM
        # iteration; profiles/r2_tuning_log.md, r3_tuning_log.md)

    CHAIN_MAX_W = 2   # widest chunk (words) the one-wave per-word chain kernel takes (csrc/hip/kernels.h kGsChain)

    @classmethod
    def wide_u_edges(cls, U: int):
        """Team sizes by CHUNK WIDTH at K > 32 and U > 32 (the c.phi-table team kernels): a team's waves
        split a chunk's W = ceil(n / U) words, so at lda-c's per-word schedule (U = 1024: W = 1 for every
        document up to 1,024 words) a 4- or 8-wave team idles all but one word slot and pays two
        workgroup barriers per word, where one wave per document refreshes in-wave with no barrier.
        Documents of <= 256 words keep the 16-lane kernel (gs_smallw: throughput); above, up to W = 4 words per
        chunk, a per-word chain of up to U refreshes per sweep runs on one wave per document with a topic per
        lane (gs_chain); four waves up to W = 16, eight beyond (never below the U = 32 edges).  K = 100 shard at
        U = 1024 (profiles/r4_tuning_log.md): fixed length edges 172.4 ms per EM iteration, (8, 64) 133.2,
        (4, 32) 107.3, (2, 16) 106.7 with the one-wave team as the first range; the 16-lane kernel's 7
        digamma/exp chains per lane cost more latency per refresh than one wave's 2 (r5g: 66.4 vs 43.1 ms)."""
        wc, w4 = cls.CHAIN_MAX_W, 16
        ec, e4 = max(256, wc * U), max(2048, w4 * U)
        return ((GS_TEAM8, e4, None), (GS_TEAM4, ec, e4), (GS_CHAIN, 256, ec), (GS_SMALL, None, 256))

    @classmethod
    def narrow_wide_u_edges(cls, U: int):
        """KS <= 32 at U > 32 (lda-c's per-word schedule at K = 20, an opt-in parity mode): the LDS-table
        kernels (gs_small, the one-wave and word-per-lane teams, gs_wsteam) cannot hold U chunk tables, so
        every document past the tiny kernel's range runs with its tables in the c.phi rows: the per-word chain
        kernel (one wave per document, a topic per lane) up to chunks of CHAIN_MAX_W words, then the 4- and
        8-wave topic-group teams (gs_team GMT) by chunk width as at KS > 32."""
        wc, w4 = cls.CHAIN_MAX_W, 16
        ec, e4 = wc * U, max(2048, w4 * U)
        return ((GS_TEAM8, e4, None), (GS_TEAM4, ec, e4), (GS_CHAIN, None, ec))

    @staticmethod
    def isolate_longest(o, m: int, xcds: int = 8):
        """Workgroup order of the team8 launch giving each of its m longest documents an XCD of its own:
        workgroup b runs on XCD b mod 8 under round-robin dispatch (a speed hint only), so slots b = x mod 8,
        x < m, stay empty (-1) after the first round.  The longest document's packed rows then have the XCD's
        L2 to themselves."""
        import numpy as np
        head, rest = list(o[:m]), list(o[m:])
        out = []
        b = 0
        while head or rest:
            if b % xcds < m:
                out.append(head.pop(0) if head else -1)
            else:
                out.append(rest.pop(0) if rest else -1)
            b += 1
        while out and out[-1] == -1:
            out.pop()
        return np.asarray(out, dtype=np.int32)
