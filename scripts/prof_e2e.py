"""cProfile of the whole ml_ops flow pipeline on a synthetic day (second run; the first warms up)."""
import cProfile
import io
import os
import pstats
import shutil
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oni_ml_amd import config as CFG  # noqa: E402
from oni_ml_amd.pipeline import run  # noqa: E402
from oni_ml_amd.synth.flow import generate_flow_day  # noqa: E402

events = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
source = sys.argv[2] if len(sys.argv) > 2 else "flow"        # flow | dns
dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
backend = "hip" if dev.type == "cuda" else "torch"
tmp = tempfile.mkdtemp(prefix="oni_prof_")
if source == "dns":
    from oni_ml_amd.synth.dns import generate_dns_day
    g = generate_dns_day(os.path.join(tmp, "in"), events=events, seed=7, files=4, n_names=max(20_000, events // 10),
                         n_clients=max(5_000, events // 40), with_edge_rows=False)
    paths = dict(dns_path=g["dns_path"], top1m=g["top1m"])
else:
    generate_flow_day(os.path.join(tmp, "in/"), events=events, seed=7)
    paths = dict(flow_path=os.path.join(tmp, "in"))
for rep in range(2):
    lp = os.path.join(tmp, f"ml{rep}")
    cfg = CFG.resolve("20160122", source, tol=1e-20 if source == "flow" else 1e-6, conf_path=None, environ={},
                      lpath=lp, backend=backend, topics=20, verbose=False, **paths)
    pr = cProfile.Profile() if rep == 1 else None
    t0 = time.perf_counter()
    if pr:
        pr.enable()
    s = run(cfg, device=dev, log=lambda *a, **k: None)
    if pr:
        pr.disable()
    print(f"rep {rep}: wall {time.perf_counter() - t0:.3f} s stages {s['stage_seconds']}", flush=True)
st = io.StringIO()
pstats.Stats(pr, stream=st).sort_stats("cumulative").print_stats(45)
print(st.getvalue())
st = io.StringIO()
pstats.Stats(pr, stream=st).sort_stats("tottime").print_stats(30)
print(st.getvalue())
shutil.rmtree(tmp, ignore_errors=True)
