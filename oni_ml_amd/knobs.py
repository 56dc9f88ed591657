"""Every environment variable the framework reads (all named ONI_*), in one registry.

Production settings live in RunConfig / the CLI (config.py); these are the process-level switches: site
paths, thread counts, memory budgets, the distributed-rehearsal modes the tests use, profiling hooks.
Every read goes through ``get``, which refuses a name missing here, and tests/test_knobs.py checks
that the source tree names no other ONI_* variable and that docs/KNOBS.md lists exactly these.
(Round 5 removed ~35 A/B switches of variants measured slower; their numbers stay in profiles/.)
"""
from __future__ import annotations

import os

KNOBS = {
    # --- site / build
    "ONI_CONF": "path of the site config (duxbay.conf; default /etc/duxbay.conf)",
    "ONI_OFFLOAD_ARCH": "GPU architecture the extensions are built for (default gfx950)",
    "ONI_PYCACHE": "0: keep Python's installed bytecode caches even when read-only (utils/pycache.py)",
    "ONI_GPUS": "scripts/ml_ops.sh: GPUs to launch one process each on under torchrun (default 1)",
    # --- host resources
    "ONI_THREADS": "host threads of the native pools: CSV/parquet ingest, the C++ LDA engine, writers "
                   "(default: min(16, the rank's CPU budget = its bound CPUs, or CPUs / LOCAL_WORLD_SIZE); "
                   "the `lda` binary: all hardware threads); set, it also turns off the per-rank CPU binding "
                   "(utils/hostres.py)",
    "ONI_SEED": "seed of the `lda` binary's random start (default 4357)",
    # --- device memory
    "ONI_CPHI_GB": "HBM budget of the per-entry c.phi rows; larger corpora run the E-step in document "
                   "windows (default: windows only past 35 % of the GPU's memory)",
    "ONI_GS_STAGE": "GB budget of the staged beta rows of the longest documents (K <= 32); 0: off "
                    "(default 4)",
    # --- E-step planning
    "ONI_GS_SPLIT_MIN": "split-document kernel plan: 'N[,g=G][,batches=B][,words=W]' -- documents longer "
                        "than N words over up to G workgroups (K > 32 default 2048; 0: off)",
    "ONI_SPLIT_MAX_BLOCKS": "cap on one split-document launch's workgroups (shared or partitioned GPUs)",
    # --- distributed
    "ONI_DIST_EXCHANGE": "class_word reduction: auto | sparse | sparse-serial | dense (sparse-serial: the "
                         "all-to-all not overlapped with the private words' suff-stats)",
    "ONI_DIST_DETERMINISTIC": "1: rank-ordered reductions; chain: the torch rehearsal engine folds the "
                              "statistics over documents in corpus order (multi-rank == one process, bitwise)",
    "ONI_DIST_BACKEND": "torch.distributed backend override (gloo: several ranks rehearsed on one GPU or CPU)",
    "ONI_DIST_FORCE_GROUP": "1: a process group even for one rank (the RCCL code paths on a one-GPU box)",
    "ONI_SHARD_CHAIN": "0: plain nnz-balanced document shards instead of the chain-aware cut",
    # --- observability / process
    "ONI_ROCTX": "1: roctx ranges per stage and EM iteration (rocprofv3 --marker-trace)",
    "ONI_PROFILE": "comma list: cprofile:FILE (the command under cProfile, stats to FILE; {rank} in FILE: the rank), table (native "
                   "ingest / writer timings on stderr)",
    "ONI_FAST_EXIT": "0: full interpreter and HIP teardown after a completed ml_ops (default: os._exit)",
    "ONI_PREFETCH": "0: do not read the day's inputs on a thread while torch imports",
    "ONI_T_SPAWN": "internal: spawn time a parent (bench.py, scripts/cold_start.py) hands a child process (the child then also writes the time of its exit call to <LPATH>/.exit_mark)",
}


def get(name: str, default=None):
    """os.environ[name] (or ``default``) for a registered knob."""
    if name not in KNOBS:
        raise KeyError(f"unregistered knob {name} (oni_ml_amd/knobs.py)")
    return os.environ.get(name, default)


def profile(token: str):
    """ONI_PROFILE's entry ``token`` (or ``token:value``): True / the value, else None."""
    for t in (get("ONI_PROFILE", "") or "").split(","):
        name, _, val = t.strip().partition(":")
        if name == token:
            return val or True
    return None


def threads(default: int = 16) -> int:
    """ONI_THREADS, else min(default, this rank's CPU budget): the CPUs bound to it (utils/hostres.py
    bind_rank), or the allowed CPUs divided by LOCAL_WORLD_SIZE."""
    v = get("ONI_THREADS")
    if v:
        return max(1, int(v))
    from .utils import hostres
    return max(1, min(default, hostres.cpu_budget()))
