"""`lda est` driver on the MI355X engine: EM run + lda-c output files + checkpoint/resume.

Reference call site: ``mpiexec -n 20 -f machinefile ./lda est 2.5 20 settings.txt 20 model.dat random <dir>``
(ml_ops.sh:80).  Outputs (README.md:116-121):

  000.beta/.other           model before the first EM iteration
  %03d.beta/.other/.gamma   every LAG=5 iterations
  final.beta/.other/.gamma  at convergence
  likelihood.dat            "%10.10f\\t%5.5e" per EM iteration
  word-assignments.dat      per-word argmax topic under the final model (lda-c writes it on every run)
  <rank>.gamma / <rank>.beta  (multi-rank runs; opt-in on one) each rank's gamma block and the log of
                            its local class_word rows over the global class totals, so
                            final.beta = log(sum_r exp(<r>.beta)) (README.md:121 "<worker index>.beta")

plus ``checkpoint.npz`` every LAG iterations (log beta, alpha, iteration,
likelihood history, VAR_MAX_ITER, RNG-free) for exact ``--resume``.
Only rank 0 writes combined files; gamma is gathered in rank order, so
final.gamma line j is corpus document j (lda_post.py pairs it with doc.dat).
"""
from __future__ import annotations

import json
import os
import queue
import threading
import time
from typing import Optional

import numpy as np
import torch

from ...corpus.csr import Corpus
from ...io import ldac
from .em import DeviceHandoff, LDAEngine, LDAResult
from .settings import LAG, LDASettings

CKPT = "checkpoint.npz"


class AsyncWriter:
    """Background threads for the LAG-period and final model files.

    lda-c writes %03d.beta/.gamma every LAG iterations inside its EM loop; here
    the host copies are handed to these threads (the C++ writers release the GIL)
    so the device keeps iterating while text is formatted.  Jobs start in
    submission order on ``workers`` threads (every job writes its own file: a text
    job's formatting overlaps another's disk write, e.g. the 3.6 GB final_model.npz
    of config 5); `close()` drains the queue and re-raises the first error."""

    def __init__(self, workers: int = 2):
        self._qs = [queue.Queue() for _ in range(workers)]
        self._err: Optional[BaseException] = None
        self._next = 0
        self._ts = [threading.Thread(target=self._loop, args=(q,), name=f"oni-lda-writer{i}", daemon=True)
                    for i, q in enumerate(self._qs)]
        for t in self._ts:
            t.start()

    def _loop(self, q):
        from ...ops import native
        from ...utils.sched import background_priority
        background_priority()
        native.background_thread_budget(len(self._qs))   # the writers share the rank's budget
        while True:
            job = q.get()
            if job is None:
                return
            if self._err is None:
                try:
                    job()
                except BaseException as e:  # surfaced by close()
                    self._err = e
            job = None      # drop the job's arrays now (pooled pinned buffers go back to the pool)

    def submit(self, fn, *args, key: Optional[str] = None, **kw):
        """``key``: jobs with the same key run on one thread in submission order (one file rewritten
        several times, e.g. checkpoint.npz); other jobs go round-robin."""
        if self._err is not None:
            raise self._err
        if key is not None:
            i = sum(key.encode()) % len(self._qs)
        else:
            i = self._next
            self._next = (self._next + 1) % len(self._qs)
        self._qs[i].put(lambda: fn(*args, **kw))

    def close(self):
        for q in self._qs:
            q.put(None)
        for t in self._ts:
            t.join()
        if self._err is not None:
            raise self._err


def _append_text(path: str, text: str):
    with open(path, "a") as f:
        f.write(text)


def _host(x):
    """A DeviceHandoff's host array (copied on the calling writer thread), dict values resolved, else x."""
    if isinstance(x, DeviceHandoff):
        return x.get()
    if isinstance(x, dict):
        return {k: _host(v) for k, v in x.items()}
    return x


def _resolved(fn):
    """fn with every DeviceHandoff argument (and dict value) replaced by its host array, in the writer thread."""
    def run(*args, **kw):
        return fn(*[_host(a) for a in args], **{k: _host(v) for k, v in kw.items()})
    return run


def _after(event, fn):
    """fn, run once ``event`` (a queued device-to-host copy of its inputs, or None) has completed."""
    if event is None:
        return fn

    def run(*args, **kw):
        event.synchronize()
        return fn(*args, **kw)
    return run


def save_checkpoint(outdir: str, eng: LDAEngine, iteration: int, L_old: float, history):
    """Collective under the sparse class_word exchange: every rank calls it (rank 0 writes)."""
    st = eng.state_arrays()
    lb = eng.log_beta(torch.from_numpy(st["cw"]).to(eng.cw.device))
    if eng.dist is not None and eng.dist.rank != 0:
        return
    _write_checkpoint(outdir, dict(log_beta=lb, alpha=np.float64(eng.alpha), iteration=np.int64(iteration),
                                   likelihood_old=np.float64(L_old), var_max_iter=np.int64(eng.var_max_iter),
                                   history=np.asarray(history, np.float64).reshape(-1, 2), **st))


def _write_checkpoint(outdir: str, arrays: dict):
    """Atomic checkpoint.npz (temp file + rename): a crash never leaves a torn checkpoint."""
    tmp = os.path.join(outdir, CKPT + ".tmp.npz")
    np.savez(tmp, **arrays)
    os.replace(tmp, os.path.join(outdir, CKPT))


def load_final(outdir: str):
    """(gamma, log_beta) of a finished run: the binary copy when present (a multi-rank run stores only
    log beta there), else the lda-c text files."""
    p = os.path.join(outdir, "final_model.npz")
    if os.path.exists(p):
        with np.load(p, allow_pickle=False) as z:
            if "gamma" in z.files:
                return z["gamma"], z["log_beta"]
            lb = z["log_beta"]
        return ldac.load_gamma(os.path.join(outdir, "final.gamma")), lb
    lb, _ = ldac.load_model(os.path.join(outdir, "final"))
    return ldac.load_gamma(os.path.join(outdir, "final.gamma")), lb


def _save_npz_atomic(path: str, **arrays):
    """np.savez to a temp name, then rename: a crash never leaves a torn or half-written file."""
    tmp = path + ".tmp.npz"
    np.savez(tmp, **arrays)
    os.replace(tmp, path)


def load_final_rows(outdir: str, d0: int, d1: int):
    """(gamma rows [d0, d1), log_beta) of a finished run, exact: from the binary copies (final_model.npz;
    a multi-rank run's per-rank final_gamma.rank<r>.npz blocks, any world size), else final.gamma's text.

    The rank blocks are used only when they come from ONE run -- the same (world size, final likelihood)
    stamp in every file, exactly `world` files -- and tile the whole corpus without gap or overlap; a
    leftover file of another run (a crash before the stage marker, resumed with fewer GPUs) makes the
    set fail that check and the text of final.gamma is read instead."""
    import glob
    runs = {}
    for f in glob.glob(os.path.join(outdir, "final_gamma.rank*.npz")):
        with np.load(f, allow_pickle=False) as z:
            if "run" not in z.files:
                continue
            world, lik = int(z["run"][0]), float(z["run"][1])
            a, b = (int(x) for x in z["doc_range"])
            runs.setdefault((world, lik), []).append((a, b, f))
    p = os.path.join(outdir, "final_model.npz")
    for (world, _), blocks in runs.items():
        if len(blocks) != world or not os.path.exists(p):
            continue
        blocks.sort(key=lambda x: x[0])
        if blocks[0][0] != 0 or any(blocks[i][1] != blocks[i + 1][0] for i in range(len(blocks) - 1)) \
                or blocks[-1][1] < d1:
            continue
        rows = []
        for a, b, f in blocks:
            if a < d1 and b > d0:
                with np.load(f, allow_pickle=False) as z:
                    rows.append(z["gamma"][max(0, d0 - a):min(b, d1) - a])
        with np.load(p, allow_pickle=False) as z:
            lb = z["log_beta"]
        K = rows[0].shape[1] if rows else lb.shape[0]
        return (np.concatenate(rows) if rows else np.zeros((0, K))), lb
    g, lb = load_final(outdir)
    return g[d0:d1], lb


def load_checkpoint(outdir: str) -> Optional[dict]:
    p = os.path.join(outdir, CKPT)
    if not os.path.exists(p):
        return None
    with np.load(p, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def estimate(corpus: Corpus, num_topics: int, alpha_init: float, settings: LDASettings, start: str, outdir: str,
             backend: str = "auto", device=None, dist=None, seed: int = 0, resume: bool = False,
             write_word_assignments: bool = False, write_rank_gamma: bool = False, verbose: bool = False,
             fault_at_iteration: Optional[int] = None, defer_files: bool = False, local_shard: bool = False,
             doc_offset: int = 0, cpu_shards: int = 1) -> LDAResult:
    """Run EM and write lda-c files.  `start`: random | seeded | <model prefix>.

    `fault_at_iteration` raises after that EM iteration (fault-injection hook for the resume tests).
    `cpu_shards` (cpu backend, one process): oni-lda-c's MPI ranks -- document shards whose statistics are
    reduced in shard order (``lda est <nproc>``).
    `defer_files`: return while the background writer is still formatting the LAG / final model
    files; the caller must call ``res.close_files()`` (which re-raises a write error, and with several
    ranks is a collective).  Without it the files are complete when this returns.
    `local_shard`: ``corpus`` is this rank's document shard starting at global document ``doc_offset``
    (the row-sharded pipeline).

    Several ranks: gamma is never gathered.  Each rank formats its own rows (``res.gamma`` = this
    rank's block) into a part file, and the parts are concatenated in rank order into
    ``<tag>.gamma`` / ``word-assignments.dat`` when the files are closed -- oni-lda-c's per-worker
    ``<rank>.gamma`` blocks "combined to form final.gamma" (README.md:121)."""
    rank0 = dist is None or dist.rank == 0
    multi = dist is not None and dist.active
    r = 0 if dist is None else dist.rank
    if rank0:
        os.makedirs(outdir, exist_ok=True)

    def _now():
        if torch.cuda.is_available() and device is not None and torch.device(device).type == "cuda":
            torch.cuda.synchronize()
        return time.perf_counter()

    t_start = _now()
    eng = LDAEngine(corpus, num_topics, settings, alpha_init=alpha_init, backend=backend, device=device, dist=dist,
                    seed=seed, local_shard=local_shard, doc_offset=doc_offset)
    if eng.backend == "cpu":
        eng.cpu_shards = max(1, int(cpu_shards))   # lda est <nproc>: the C++ engine's document shards
    timing = dict(setup_s=round(_now() - t_start, 4))
    parts = []          # (final file, this rank's part file): concatenated at close
    start_it, L_old, hist = 0, 0.0, []
    ck = load_checkpoint(outdir) if resume else None
    if ck is not None:
        if "cw" in ck and tuple(ck["cw"].shape) == tuple(eng.cw.shape):
            eng.load_state_arrays(ck["cw"], ck["class_total"], float(ck["alpha"]))
        else:
            eng.init_from_model(ck["log_beta"], float(ck["alpha"]))
        eng.var_max_iter = int(ck["var_max_iter"])
        start_it, L_old = int(ck["iteration"]), float(ck["likelihood_old"])
        hist = [tuple(x) for x in ck["history"].tolist()]
        mode = "resume"
        if rank0:  # likelihood.dat holds exactly the checkpointed iterations
            with open(os.path.join(outdir, "likelihood.dat"), "w") as f:
                for L, c in hist:
                    f.write(ldac.format_likelihood_line(L, c))
    elif start in ("random", "seeded"):
        mode = start
        if rank0:
            open(os.path.join(outdir, "likelihood.dat"), "w").close()
    else:
        lb, a = ldac.load_model(start)
        eng.init_from_model(lb, a)
        mode = "resume"
        if rank0:
            open(os.path.join(outdir, "likelihood.dat"), "w").close()

    history = list(hist)

    writer = AsyncWriter()
    lik_path = os.path.join(outdir, "likelihood.dat")
    lik_lines = []      # likelihood.dat lines not yet handed to the writer

    def flush_likelihood():
        # appended by the writer thread (one file, one key: in order), not by the thread driving the GPU:
        # an open/append/close per EM iteration waited on the filesystem behind the lda_pre text files
        # (profiles/r6_lda_stage.md); a resume rewrites the file from the checkpoint's history anyway
        if rank0 and lik_lines:
            text = "".join(lik_lines)
            lik_lines.clear()
            writer.submit(_append_text, lik_path, text, key="likelihood")

    def on_iteration(e, i, lik, conv):
        history.append((lik, conv))
        if rank0:
            lik_lines.append(ldac.format_likelihood_line(lik, conv))
        if fault_at_iteration is not None and i >= fault_at_iteration:
            flush_likelihood()
            raise RuntimeError(f"injected fault after EM iteration {i}")
    # this rank's exact gamma block of an earlier run (load_final_rows) is stale from here on
    stale = os.path.join(outdir, f"final_gamma.rank{r}.npz")
    if os.path.exists(stale):
        os.remove(stale)

    saved = {}          # the final save's host copies, reused for the result

    def on_save(tag, e):
        flush_likelihood()
        # collectives first, on every rank: global class_word (sparse exchange)
        ckpt = tag not in ("000", "final")
        cwg = e.global_cw()
        ev_st = None
        st = None
        # LAG saves take their pinned buffers from the process's pool (the writer's jobs are their only
        # users); the final save's arrays are returned to the caller and get fresh ones
        reuse = tag != "final"
        ho = e.save_handoff(cwg, gamma=tag != "000", checkpoint=ckpt) if reuse and not multi else None
        if ho is not None:
            # one rank on the GPU: device copies + one event here, the host copies on the writer threads
            if not rank0:
                return
            writer.submit(_resolved(ldac.save_model), os.path.join(outdir, tag), ho["log_beta"], e.alpha)
            if "gamma" in ho:
                writer.submit(_resolved(ldac.save_gamma), os.path.join(outdir, f"{tag}.gamma"), ho["gamma"])
            if ckpt:
                ck = dict(log_beta=ho["log_beta"], alpha=np.float64(e.alpha), iteration=np.int64(int(tag)),
                          likelihood_old=np.float64(history[-1][0] if history else 0.0),
                          var_max_iter=np.int64(e.var_max_iter),
                          history=np.asarray(history, np.float64).reshape(-1, 2),
                          cw=ho["cw"], class_total=ho["class_total"])
                writer.submit(_resolved(_write_checkpoint), outdir, ck, key="checkpoint")
            return
        if ckpt:   # the checkpoint's exact statistics, copied behind the device work like the model
            cw_h, _ = e.host_copy_deferred(cwg, reuse=reuse)
            ct_h, ev_st = e.host_copy_deferred(e.class_total, reuse=reuse)   # queued after cw: its event covers both
            st = dict(cw=cw_h, class_total=ct_h)
        # host copies queued behind the device work; the writer waits for their events
        lb, ev_lb = e.log_beta_deferred(cwg, reuse=reuse)
        g, ev_g = e.local_gamma_deferred(reuse=reuse) if tag != "000" else (None, None)
        if tag == "final":
            for ev in (ev_lb, ev_g):
                if ev is not None:
                    ev.synchronize()
            ev_lb = ev_g = None
            saved.update(log_beta=lb, gamma=g)
        if g is not None and multi:
            part = os.path.join(outdir, f".{tag}.gamma.part{r}")
            parts.append((os.path.join(outdir, f"{tag}.gamma"), part))
            writer.submit(_after(ev_g, ldac.save_gamma), part, g)
        if multi and tag == "final":
            # exact binary gamma rows of this rank's documents (a resumed lda_post reads them instead of the
            # %5.10f text of final.gamma, load_final_rows)
            d0, d1 = e.doc_range
            run = np.asarray([dist.world_size, history[-1][0] if history else 0.0], np.float64)
            writer.submit(_save_npz_atomic, os.path.join(outdir, f"final_gamma.rank{r}.npz"), gamma=g,
                          doc_range=np.asarray([d0, d1], np.int64), run=run)
        if write_rank_gamma and tag == "final":
            writer.submit(ldac.save_gamma, os.path.join(outdir, f"{r}.gamma"), g)
            writer.submit(ldac.save_beta, os.path.join(outdir, f"{r}.beta"), e.local_log_beta())
        if not rank0:
            return
        writer.submit(_after(ev_lb, ldac.save_model), os.path.join(outdir, tag), lb, e.alpha)
        if g is not None and not multi:
            writer.submit(_after(ev_g, ldac.save_gamma), os.path.join(outdir, f"{tag}.gamma"), g)
        if tag not in ("000", "final"):
            # engine state is read now (host copies); only the file write is deferred
            ck = dict(log_beta=lb, alpha=np.float64(e.alpha), iteration=np.int64(int(tag)),
                      likelihood_old=np.float64(history[-1][0] if history else 0.0),
                      var_max_iter=np.int64(e.var_max_iter), history=np.asarray(history, np.float64).reshape(-1, 2),
                      **st)
            writer.submit(_after(ev_st, _after(ev_lb, _write_checkpoint)), outdir, ck, key="checkpoint")
        if tag == "final":  # exact binary copy of what final.* hold as text (stage resume reloads this)
            extra = {} if multi else dict(gamma=g)
            writer.submit(np.savez, os.path.join(outdir, "final_model.npz"), log_beta=lb,
                          alpha=np.float64(e.alpha), **extra)

    def concat_parts():
        if multi:
            from ...parallel import shardio as SIO
            for path, part in parts:
                SIO.concat_part_files(dist, path, part)
        parts.clear()

    def close_files():
        writer.close()
        concat_parts()

    # error path (StageRunner.finish_deferred(suppress=True)): only the failing rank may get there, so
    # drain this rank's writer and leave the collective part-file concatenation out
    close_files.abort = writer.close

    ok = False
    try:
        # corpus_global: only when every rank holds the whole corpus (seeded init draws from it)
        res = eng.run(start=mode, corpus_global=None if local_shard else corpus, on_iteration=on_iteration,
                      on_save=on_save, start_iteration=start_it, likelihood_old=L_old, verbose=verbose and rank0)
        ok = True
    finally:
        if not (ok and defer_files):
            writer.close()
    timing["em_s"] = round(res.seconds, 4)
    # where the GPU-driving thread spent the EM loop (em.py _hphase): init, enqueue, wait, save, save_final
    timing["em_host"] = {k: round(v, 4) for k, v in getattr(eng, "host_phases", {}).items()}
    t_out = _now()
    res.likelihoods = history
    # this rank's documents (all of them with one rank); the final save already copied both
    res.log_beta = saved["log_beta"] if "log_beta" in saved else eng.log_beta()
    res.gamma = saved["gamma"] if saved.get("gamma") is not None else eng.local_gamma()
    res.doc_range = eng.doc_range
    timing["model_copies_s"] = round(_now() - t_out, 4)
    if write_word_assignments:
        # run_em's final pass: a fresh E-step under the final model (after gamma and beta were read),
        # the argmax of each word's phi; native formatting on the background writer with the deferred
        # model files when allowed (the caller's next stages do not wait for it)
        wa, shard = os.path.join(outdir, "word-assignments.dat"), eng.corpus
        t_wa = _now()
        z = eng.word_assignments()
        timing["final_pass_s"] = round(_now() - t_wa, 4)
        if multi:
            part = os.path.join(outdir, f".word-assignments.dat.part{r}")
            parts.append((wa, part))
            wa = part

        def _assign():
            _write_assignment_file(wa, shard, z)

        if defer_files:
            writer.submit(_assign)
        else:
            _assign()
    if not defer_files:
        concat_parts()
    res.close_files = close_files if defer_files else (lambda: None)
    timing["total_s"] = round(_now() - t_start, 4)
    res.timing = timing
    nnz = dist.allreduce_int(eng.corpus.nnz) if multi else eng.corpus.nnz
    if rank0:
        with open(os.path.join(outdir, "lda_stats.json"), "w") as f:
            json.dump(dict(em_iterations=res.em_iterations, seconds=res.seconds, alpha=res.alpha,
                           backend=eng.backend, docs=eng.global_docs, terms=eng.V, nnz=nnz, ranks=dist.world_size
                           if multi else 1, timing=timing, metrics=eng.metrics(res.seconds, res.em_iterations),
                           per_iter=[s.__dict__ for s in res.stats]), f)
    res.engine = eng
    return res


def word_topics(corpus: Corpus, log_beta: np.ndarray, gamma: np.ndarray, device=None,
                chunk: int = 1 << 22) -> np.ndarray:
    """Per corpus entry argmax_k (psi(gamma_dk) + log beta_{k,w}) as int64 [nnz] (first maximum on ties).

    The argmax of phi_nk ~ exp(psi(gamma_k)) beta_{k,w} (lda-c write_word_assignment); evaluated on
    the engine's device in chunks of ``chunk`` entries ([chunk, K] doubles at a time)."""
    from .special import digamma
    dev = torch.device(device) if device is not None else torch.device("cpu")
    psi = digamma(torch.from_numpy(np.ascontiguousarray(gamma, np.float64)).to(dev))       # [D, K]
    lbt = torch.from_numpy(np.ascontiguousarray(log_beta.T, np.float64)).to(dev)           # [V, K]
    lens = torch.from_numpy(corpus.lengths().astype(np.int64)).to(dev)
    doc_of = torch.repeat_interleave(torch.arange(corpus.num_docs, device=dev), lens)
    w = torch.from_numpy(corpus.word_idx.astype(np.int64)).to(dev)
    z = torch.empty(corpus.nnz, dtype=torch.int64, device=dev)
    for a in range(0, corpus.nnz, chunk):
        b = min(corpus.nnz, a + chunk)
        z[a:b] = torch.argmax(psi[doc_of[a:b]] + lbt[w[a:b]], dim=1)
    return z.cpu().numpy()


def write_assignments(path: str, corpus: Corpus, log_beta: np.ndarray, gamma: np.ndarray, device=None):
    """word-assignments.dat: per doc ``%03d`` length then `` %04d:%02d`` word:argmax-topic
    (lda-c write_word_assignment), formatted by the multithreaded native corpus writer."""
    _write_assignment_file(path, corpus, word_topics(corpus, log_beta, gamma, device))


def _write_assignment_file(path: str, corpus: Corpus, z: np.ndarray):
    from ...ops import native
    native.lib().write_ldac_corpus(path, corpus.doc_ptr, corpus.word_idx, z, assignments=True)


def write_assignments_reference(path: str, corpus: Corpus, log_beta: np.ndarray, gamma: np.ndarray):
    """Literal per-document loop (test oracle for write_assignments)."""
    from .special import digamma
    psi = digamma(gamma)
    with open(path, "w") as f:
        for d in range(corpus.num_docs):
            a, b = corpus.doc_ptr[d], corpus.doc_ptr[d + 1]
            w = corpus.word_idx[a:b]
            z = np.argmax(psi[d][None, :] + log_beta[:, w].T, axis=1)
            f.write("%03d" % (b - a) + "".join(" %04d:%02d" % (wi, zi) for wi, zi in zip(w.tolist(), z.tolist())) + "\n")
