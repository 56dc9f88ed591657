"""Command line: ``python -m oni_ml_amd <command> ...`` (and scripts/ml_ops.sh).

  ml_ops YYYYMMDD {flow|dns} [TOL] [options]   end-to-end run (reference ml_ops.sh:1-123)
  lda est <alpha> <k> <settings> <nproc> <corpus> <random|seeded|prefix> <dir>
                                               oni-lda-c command line (ml_ops.sh:80) on the MI355X engine
  lda inf <settings> <model-prefix> <corpus> <name>
  lda_pre <LPATH>/                             lda_pre.py equivalent (doc_wc.dat -> words/doc/model.dat)
  lda_post <LPATH>/                            lda_post.py equivalent (final.* -> doc/word_results.csv)
  synth {flow|dns} --out DIR ...               synthetic inputs (flow CSV day, DNS parquet, top-1m.csv)
  qtiles [show] <flow_qtiles>                  print cuts of the legacy qtiles format
  qtiles gen <FLOW_PATH> [--out DIR]           gen_qtiles.sh + qtiles.py: sample ntile cuts -> flow_qtiles
  install [--nodes a,b] [--dry-run]            install_ml.sh: rsync the framework to NODES:${LUSER}/ml

Multi-GPU: launch with torchrun (one process per GPU).  Every ml_ops stage is row-sharded over the ranks
(pipeline/sharded.py): each featurizes its byte range of the day, builds and trains its document shard and
scores its own rows; they meet only in tensor collectives over RCCL (parallel/shardio.py, parallel/dist.py).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import time

from . import knobs

# wall-clock marks (time.time()) of the process's start-up: `python -m oni_ml_amd` records "main" before its
# first import; ml_ops adds the rest.  ONI_T_SPAWN (set by a parent that launches this process, e.g. bench.py's
# cold run) is the spawn time, so interpreter start-up is measured too (startup_marks in run_summary.json).
MARKS = {}
# set by a completed ml_ops when ONI_FAST_EXIT (default 1) allows `python -m oni_ml_amd` to skip teardown
FAST_EXIT = False
# <LPATH>/.exit_mark when a timing parent set ONI_T_SPAWN: __main__ writes the time of its exit call there
EXIT_MARK = None


def _tool_attached() -> bool:
    """A profiler, tracer or coverage tool that writes its output at exit (python -m cProfile / coverage,
    rocprofv3's preloaded tool library): the process then keeps the normal teardown."""
    if sys.getprofile() is not None or sys.gettrace() is not None:
        return True
    if "coverage" in sys.modules or "cProfile" in sys.modules:
        return True
    pre = os.environ.get("LD_PRELOAD", "")
    return "rocprof" in pre or any(k.startswith(("ROCP_", "ROCPROF")) for k in os.environ)


def startup_marks() -> dict:
    """Seconds from the spawn (ONI_T_SPAWN, else "main") to each recorded mark."""
    t0 = float(knobs.get("ONI_T_SPAWN", MARKS.get("main", 0.0)) or 0.0)
    return {k: round(v - t0, 4) for k, v in sorted(MARKS.items(), key=lambda kv: kv[1])} if t0 else {}


SYNTAX = """ml_ops.sh syntax error
Please run ml_ops.sh again with the correct syntax:
./ml_ops.sh YYYYMMDD TYPE [TOL]
for example:
./ml_ops.sh 20160122 dns 1e-6
./ml_ops.sh 20160122 flow"""


def _common_lda_args(ap):
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch", "cpu"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--gs-updates", type=int, default=None,
                    help="U, gamma refreshes per document sweep of the fp64 GPU engine (default 32; up to 4096 "
                         "at K > 32; lda-c's per-word schedule is U >= document length; -1: the U per K that "
                         "meets lda-c parity, profiles/r3_precision_parity.md)")
    ap.add_argument("--lag", type=int, default=None, help="period of the %%03d model files (lda-c: 5; 0: only 000 "
                                                          "and final)")
    ap.add_argument("--cphi-gb", type=float, default=None,
                    help="HBM budget of the per-entry c.phi rows: larger corpora run the E-step in document windows")


def _apply_lda_args(a, st):
    """--gs-updates / --lag / --cphi-gb onto an LDASettings (and the engine's environment)."""
    if a.gs_updates is not None:
        st.gs_updates = int(a.gs_updates)
    if a.lag is not None:
        st.lag = int(a.lag)
    if a.cphi_gb is not None:
        os.environ["ONI_CPHI_GB"] = str(a.cphi_gb)
    return st


def clean_workdir(lpath: str):
    """ml_ops.sh:53-54: remove stale *.dat,*.beta,*.gamma,*.other,*.pkl; keep *.csv (analyst feedback)."""
    for pat in ("*.dat", "*.beta", "*.gamma", "*.other", "*.pkl", "checkpoint.npz", "final_model.npz",
                "final_gamma.rank*.npz"):
        for f in glob.glob(os.path.join(lpath, pat)):
            os.unlink(f)
    shutil.rmtree(os.path.join(lpath, ".stages"), ignore_errors=True)


def cmd_ml_ops(argv):
    ap = argparse.ArgumentParser(prog="ml_ops", description="suspicious-connects end-to-end run")
    ap.add_argument("fdate", nargs="?", default="")
    ap.add_argument("dsource", nargs="?", default="")
    ap.add_argument("tol", nargs="?", default=None)
    ap.add_argument("--conf", default=knobs.get("ONI_CONF", "/etc/duxbay.conf"))
    ap.add_argument("--lpath")
    ap.add_argument("--flow-path")
    ap.add_argument("--dns-path")
    ap.add_argument("--top1m")
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--alpha", type=float, default=2.5)
    ap.add_argument("--settings", help="lda-c settings.txt (default: upstream lda-c defaults)")
    ap.add_argument("--dupfactor", type=int)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--compat", default="strict", choices=["strict", "fixed"])
    ap.add_argument("--start", default="random")
    ap.add_argument("--resume", action="store_true")
    ap.add_argument("--keep-doc-wc", action="store_true", help="keep doc_wc.dat (the reference deletes it)")
    ap.add_argument("--word-assignments", dest="word_assignments", action="store_true", default=True,
                    help="write word-assignments.dat (default, as lda-c does on every run)")
    ap.add_argument("--no-word-assignments", dest="word_assignments", action="store_false")
    ap.add_argument("--rank-gamma", action="store_true", default=None,
                    help="write <rank>.gamma / <rank>.beta per GPU (default: on when running on several GPUs and K x V <= 2^26)")
    ap.add_argument("--threads", type=int, default=None,
                    help="host threads of the stage pools (default: min(8, this rank's CPU budget))")
    ap.add_argument("--deliver", action="store_true", help="scp -r LPATH UINODE:RPATH (ml_ops.sh:121)")
    ap.add_argument("--cuts", help="fixed flow cuts: a flow_qtiles file or its text (the reference's CUT)")
    ap.add_argument("--hdfs", action="store_true",
                    help="stage hdfs:// inputs locally and publish results to HPATH (ml_ops.sh HDFS steps)")
    ap.add_argument("--hadoop", default="hadoop", help="hadoop CLI for --hdfs")
    ap.add_argument("--quiet", action="store_true")
    _common_lda_args(ap)
    a = ap.parse_args(argv)
    if len(a.fdate) != 8 or not a.dsource:
        print(SYNTAX)
        return 1
    # (a HIP context created on a thread during `import torch`, and a warm-up thread launching the first
    # stages' kernels while the inputs parse, were both measured slower and removed in round 5:
    # profiles/r4_cold_start.md, profiles/r4_tuning_log.md §3)
    from . import config as CFG

    def resolve(world):
        return CFG.resolve(a.fdate, a.dsource, tol=float(a.tol) if a.tol is not None else None, conf_path=a.conf,
                           lpath=a.lpath, flow_path=a.flow_path, dns_path=a.dns_path, top1m=a.top1m,
                           topics=a.topics, alpha=a.alpha, dupfactor=a.dupfactor, gpus=world, backend=a.backend,
                           compat=a.compat, seed=a.seed, start=a.start, resume=a.resume, threads=a.threads,
                           write_doc_wc=a.keep_doc_wc, word_assignments=a.word_assignments,
                           rank_gamma=a.rank_gamma, verbose=not a.quiet, cuts=a.cuts, hdfs=a.hdfs or None,
                           hadoop=a.hadoop)
    # one process, fresh run: the day's inputs are read on a thread while torch imports
    # (pipeline/prefetch.py); the load stage takes the result
    from .pipeline import prefetch
    if (knobs.get("ONI_PREFETCH", "1") != "0" and a.gpus <= 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1
            and not a.resume and not a.hdfs):
        try:
            prefetch.start_for(resolve(1), fork=not _tool_attached(), after_import=True)
        except Exception:  # noqa: BLE001 -- a bad configuration is reported by the resolve below
            pass
    try:
        return _ml_ops_body(a, resolve)
    finally:
        prefetch.drop_all()   # a run that failed before its load stage: no forked child or /dev/shm files left


def _ml_ops_body(a, resolve):
    import torch  # noqa: F401  (its import time is a start-up mark of its own)
    MARKS["torch_imported"] = time.time()
    from .pipeline import prefetch
    prefetch.imported()
    from .models.lda.settings import LDASettings
    from .parallel import dist as D
    MARKS["package_imported"] = time.time()

    ctx = D.init_from_env(expected_world=a.gpus if a.gpus > 1 else None)
    if ctx.device.type == "cuda":
        import torch
        torch.zeros(1, device=ctx.device)     # HIP runtime + context (the first device call)
    MARKS["device_ready"] = time.time()
    cfg = resolve(ctx.world_size)
    if a.settings:
        cfg.settings = LDASettings.load(a.settings)
    _apply_lda_args(a, cfg.settings)
    cfg.validate()
    from .pipeline import run
    from .pipeline.runner import RunLock
    log = (lambda *x, **k: None) if (a.quiet or ctx.rank != 0) else print
    t0 = time.perf_counter()
    lock = None
    if ctx.rank == 0:
        os.makedirs(cfg.lpath, exist_ok=True)
        if not cfg.resume:
            clean_workdir(cfg.lpath)
        lock = RunLock(os.path.join(cfg.lpath, ".lock")).__enter__()
    ctx.barrier()
    MARKS["pipeline_start"] = time.time()
    try:
        summary = run(cfg, dist=ctx if ctx.active else None, device=ctx.device, log=log)
    finally:
        if lock is not None:
            lock.__exit__(None, None, None)
    MARKS["pipeline_end"] = time.time()
    if ctx.rank == 0:
        summary["wall_seconds"] = time.perf_counter() - t0
        summary["startup_marks"] = startup_marks()
        with open(os.path.join(cfg.lpath, "run_summary.json"), "w") as f:
            json.dump(summary, f, indent=1, default=str)
        log(json.dumps(summary, default=str))
        if a.deliver:
            ui, rp = cfg.extra.get("UINODE"), cfg.extra.get("RPATH")
            if ui and rp:
                subprocess.run(["scp", "-r", cfg.lpath, f"{ui}:{rp}"], check=True)
    ctx.shutdown()
    global FAST_EXIT, EXIT_MARK
    FAST_EXIT = knobs.get("ONI_FAST_EXIT", "1") != "0" and not _tool_attached()
    if ctx.rank == 0 and knobs.get("ONI_T_SPAWN", ""):
        EXIT_MARK = os.path.join(cfg.lpath, ".exit_mark")
    return 0


def cmd_lda(argv):
    if not argv or argv[0] not in ("est", "inf"):
        print("usage: lda est [initial alpha] [k] [settings] [nproc] [data] [random/seeded/*] [directory]\n"
              "       lda inf [settings] [model] [data] [name]")
        return 1
    from .io import ldac
    from .models.lda.settings import LDASettings
    if argv[0] == "est":
        ap = argparse.ArgumentParser(prog="lda est")
        for n in ("alpha", "k", "settings", "nproc", "data", "start", "directory"):
            ap.add_argument(n)
        ap.add_argument("--resume", action="store_true")
        ap.add_argument("--word-assignments", dest="word_assignments", action="store_true", default=True)
        ap.add_argument("--no-word-assignments", dest="word_assignments", action="store_false")
        _common_lda_args(ap)
        a = ap.parse_args(argv[1:])
        from .models.lda.estimate import estimate
        from .parallel import dist as D
        try:
            nproc = int(a.nproc)
        except ValueError:
            nproc = 0
        if nproc < 1:
            print(f"lda est: nproc must be a positive rank count, got {a.nproc!r}", file=sys.stderr)
            return 1
        world = int(os.environ.get("WORLD_SIZE", "1"))
        # oni-lda-c's nproc is its MPI rank count (ml_ops.sh:80 passes PROCESS_COUNT = 20).  Here the ranks are
        # the torchrun processes (one per GPU): a multi-rank launch must say how many it is; one process runs
        # every document (on the GPU, or the C++ engine with nproc document shards reduced in shard order --
        # the MPI job's arithmetic)
        if world > 1 and nproc != world:
            print(f"lda est: nproc = {nproc} but {world} ranks were launched (WORLD_SIZE); pass nproc = {world}",
                  file=sys.stderr)
            return 1
        ctx = D.init_from_env()
        corpus = ldac.read_model_dat(a.data)
        st = _apply_lda_args(a, LDASettings.load(a.settings))
        if world == 1 and nproc > 1 and a.backend not in ("cpu",) and ctx.device.type == "cuda":
            print(f"lda est: nproc = {nproc}: one process runs every document on one GPU (launch nproc processes "
                  f"with torchrun --nproc-per-node for that many GPUs)", file=sys.stderr)
        res = estimate(corpus, int(a.k), float(a.alpha), st, a.start, a.directory, backend=a.backend,
                       device=ctx.device, dist=ctx if ctx.active else None, seed=a.seed, resume=a.resume,
                       write_word_assignments=a.word_assignments, verbose=True,
                       cpu_shards=nproc if world == 1 else 1)
        if ctx.rank == 0:
            print(f"em iterations: {res.em_iterations}  seconds: {res.seconds:.3f}")
        ctx.shutdown()
        return 0
    ap = argparse.ArgumentParser(prog="lda inf")
    for n in ("settings", "model", "data", "name"):
        ap.add_argument(n)
    _common_lda_args(ap)
    a = ap.parse_args(argv[1:])
    from .models.lda.inference import infer_files
    infer_files(a.settings, a.model, a.data, a.name, backend=a.backend)
    return 0


def cmd_lda_pre(argv):
    """lda_pre.py <LPATH>/ : doc_wc.dat -> words.dat, doc.dat, model.dat."""
    rpath = argv[0]
    from .corpus.builder import lda_pre, read_doc_wc
    from .pipeline.common import write_corpus_files
    dwc, ips, words = read_doc_wc(os.path.join(rpath, "doc_wc.dat"))
    built = lda_pre(dwc)
    write_corpus_files(rpath, built, [ips[i] for i in built.doc_keys.tolist()], [words[i] for i in built.word_keys.tolist()])
    print(f"docs {built.corpus.num_docs} words {built.corpus.num_terms} entries {built.corpus.nnz}")
    return 0


def cmd_lda_post(argv):
    """lda_post.py <LPATH>/ : final.gamma + final.beta + doc.dat + words.dat -> doc/word_results.csv."""
    ap = argparse.ArgumentParser(prog="lda_post")
    ap.add_argument("rpath")
    ap.add_argument("--compat", default="strict", choices=["strict", "fixed"])
    a = ap.parse_args(argv)
    from .export import lda_post
    from .io import ldac
    r = a.rpath
    gamma = ldac.load_gamma(os.path.join(r, "final.gamma"))
    lb = ldac.load_beta(os.path.join(r, "final.beta"))
    lda_post.export(ldac.read_index_file(os.path.join(r, "doc.dat")), gamma, ldac.read_index_file(os.path.join(r, "words.dat")),
                    lb, os.path.join(r, "doc_results.csv"), os.path.join(r, "word_results.csv"), strict=a.compat == "strict")
    return 0


def cmd_synth(argv):
    ap = argparse.ArgumentParser(prog="synth")
    ap.add_argument("kind", choices=["flow", "dns"])
    ap.add_argument("--out", required=True)
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--files", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    if a.kind == "flow":
        from .synth.flow import generate_flow_day
        print(generate_flow_day(a.out, a.events, a.seed, files=a.files))
    else:
        from .synth.dns import generate_dns_day
        print(generate_dns_day(a.out, a.events, a.seed, files=a.files))
    return 0


def cmd_qtiles(argv):
    """qtiles show <flow_qtiles>  |  qtiles gen <FLOW_PATH> [--out DIR] [--sample-rows N] [--keep-tsv]

    gen = gen_qtiles.sh + qtiles.py: per input file the first N data rows stand in
    for Hive's TABLESAMPLE(N ROWS); ibyt deciles, ipkt ntile(3), time deciles -> qtiles.tsv ->
    <out>/flow_qtiles (consumable by ml_ops --cuts / the CUT variable)."""
    if argv and argv[0] == "gen":
        ap = argparse.ArgumentParser(prog="qtiles gen")
        ap.add_argument("flow_path")
        ap.add_argument("--out", default=".")
        ap.add_argument("--sample-rows", type=int, default=100)
        ap.add_argument("--keep-tsv", action="store_true", help="keep qtiles.tsv (gen_qtiles.sh deletes it)")
        a = ap.parse_args(argv[1:])
        import numpy as np
        from .features.flow import list_inputs
        from .features.quantiles import gen_qtiles_tsv, qtiles_from_tsv
        cols = {4: [], 5: [], 16: [], 17: []}          # hour, minute, ipkt, ibyt (27-column flow CSV)
        for path in list_inputs(a.flow_path):
            with open(path) as f:
                header = f.readline()
                n = 0
                for line in f:
                    if line == header:
                        continue
                    parts = line.rstrip("\n").split(",")
                    if len(parts) != 27:
                        continue
                    try:
                        vals = {c: float(parts[c]) for c in cols}
                    except ValueError:
                        continue
                    for c, v in vals.items():
                        cols[c].append(v)
                    n += 1
                    if n >= a.sample_rows:
                        break
        tsv = gen_qtiles_tsv(np.asarray(cols[17]), np.asarray(cols[16]), np.asarray(cols[4]), np.asarray(cols[5]))
        os.makedirs(a.out, exist_ok=True)
        if a.keep_tsv:
            with open(os.path.join(a.out, "qtiles.tsv"), "w") as f:
                f.write(tsv)
        out = os.path.join(a.out, "flow_qtiles")
        with open(out, "w") as f:
            f.write(qtiles_from_tsv(tsv))
        print(out)
        return 0
    from .features.quantiles import parse_qtiles
    path = argv[1] if argv and argv[0] == "show" else argv[0]
    with open(path) as f:
        q = parse_qtiles(f.read())
    print(json.dumps({k: v.tolist() for k, v in q.items()}))
    return 0


def cmd_install(argv):
    """install_ml.sh: rsync the framework (dot-files excluded) to every node in NODES:${LUSER}/ml."""
    ap = argparse.ArgumentParser(prog="install")
    ap.add_argument("--conf", default=knobs.get("ONI_CONF", "/etc/duxbay.conf"))
    ap.add_argument("--nodes", help="comma-separated node list (default: NODES from the config)")
    ap.add_argument("--luser", help="remote base dir (default: LUSER from the config)")
    ap.add_argument("--src", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap.add_argument("--dry-run", action="store_true", help="print the rsync commands only")
    a = ap.parse_args(argv)
    from . import config as CFG
    cfg = CFG.resolve("00000000", "flow", conf_path=a.conf)
    nodes = a.nodes.split(",") if a.nodes else cfg.extra.get("NODES") or []
    if isinstance(nodes, str):
        nodes = nodes.split()
    luser = a.luser or cfg.extra.get("LUSER")
    if not nodes or not luser:
        print("install: NODES and LUSER are required (config or --nodes/--luser)", file=sys.stderr)
        return 1
    for d in nodes:
        cmd = ["rsync", "-v", "-a", "--exclude=.*", a.src.rstrip("/") + "/", f"{d}:{luser}/ml"]
        print(" ".join(cmd))
        if not a.dry_run:
            subprocess.run(cmd, check=True)
    return 0


COMMANDS = dict(ml_ops=cmd_ml_ops, lda=cmd_lda, lda_pre=cmd_lda_pre, lda_post=cmd_lda_post, synth=cmd_synth,
                qtiles=cmd_qtiles, install=cmd_install)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] not in COMMANDS:
        print(__doc__)
        return 1
    prof = knobs.profile("cprofile")
    if isinstance(prof, str):
        prof = prof.replace("{rank}", os.environ.get("RANK", "0"))   # one file per rank under torchrun
        # host profile of a whole command (cold-start analysis, scripts/cold_start.py)
        import cProfile
        pr = cProfile.Profile()
        try:
            return pr.runcall(COMMANDS[argv[0]], argv[1:])
        finally:
            pr.dump_stats(prof)
    return COMMANDS[argv[0]](argv[1:])


if __name__ == "__main__":
    sys.exit(main())
