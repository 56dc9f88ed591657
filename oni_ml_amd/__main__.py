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
        with open(cli.EXIT_MARK, "w") as f:
            f.write(repr(time.time()))
    os._exit(rc or 0)
sys.exit(rc)
