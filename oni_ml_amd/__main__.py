import sys
import time

_T_MAIN = time.time()      # process-level start marks (cli.startup_marks): before any package import

from . import cli  # noqa: E402

cli.MARKS["main"] = _T_MAIN
cli.MARKS["cli_imported"] = time.time()
sys.exit(cli.main())
