import sys
import time

_T_MAIN = time.time()      # process-level start marks (cli.startup_marks): before any package import

from .utils import pycache  # noqa: E402

pycache.enable()           # before anything imports torch (utils/pycache.py)

from . import cli  # noqa: E402

cli.MARKS["main"] = _T_MAIN
cli.MARKS["cli_imported"] = time.time()
rc = cli.main()
if cli.FAST_EXIT:
    # ml_ops finished: every output file is closed and the process group is gone.  Leave without the
    # interpreter's and the HIP runtime's teardown (~0.5 s of a cold run's wall, profiles/r4_cold_start.md);
    # ONI_FAST_EXIT=0 keeps the full teardown
    import os
    sys.stdout.flush()
    sys.stderr.flush()
    if cli.EXIT_MARK:   # a timing parent (ONI_T_SPAWN): wall-clock time of the exit call, the rest is teardown
        t_exit = time.time()
        st = {}
        try:
            with open("/proc/self/status") as f:
                st = {k: v.split()[0] for k, v in (ln.split(":", 1) for ln in f if ":" in ln)
                      if k in ("VmRSS", "VmHWM", "RssAnon", "RssFile", "RssShmem", "VmPin", "Threads")}
        except OSError:
            pass
        with open(cli.EXIT_MARK, "w") as f:
            f.write(repr(t_exit) + " " + " ".join(f"{k}={v}" for k, v in sorted(st.items())))
    os._exit(rc or 0)
sys.exit(rc)
