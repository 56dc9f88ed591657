#!/usr/bin/env python
"""BASELINE config 5 at its real scale: a month of netflow (~100M events, 30 part files) through the
full flow pipeline (ingest -> featurize -> lda_pre -> LDA K=100 fp64 -> lda_post -> flow_post) on
the GPUs of one node.

The month is generated on the spot (synth/flow.py, chunked: one part file per day, each from its
own random stream, the address pool scaled with the event count), then the pipeline runs exactly as
`python -m oni_ml_amd.cli YYYYMMDD flow` would.  Prints one progress line per stage and writes a JSON
record (stage seconds, corpus shape, ms per EM iteration, peak HBM, ingest rate) to --out.

EM runs to lda-c's convergence test (1e-4) or `--em-iters`.  K != 20 needs compat=fixed (the
reference's lda_post.py hard-codes 20 topics).

    python scripts/config5.py --events 100000000 --days 30 --topics 100 --out gpurun_out/c5.json
"""
import argparse
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _du(path):
    return sum(os.path.getsize(os.path.join(d, f)) for d, _, fs in os.walk(path) for f in fs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, default=100_000_000)
    ap.add_argument("--days", type=int, default=30)
    ap.add_argument("--topics", type=int, default=100)
    ap.add_argument("--em-iters", type=int, default=100)
    ap.add_argument("--lag", type=int, default=0, help="LAG save period (lda-c: 5; 0 = 000 and final only)")
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--workdir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "oni_config5"))
    ap.add_argument("--out", default="gpurun_out/config5.json")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--gs-updates", type=int, default=0, help="U of the fp64 engine (0: 32)")
    ap.add_argument("--cphi-gb", type=float, default=None,
                    help="HBM budget of the engine's c.phi rows (ONI_CPHI_GB): E-step in document windows")
    a = ap.parse_args()
    if a.cphi_gb is not None:
        os.environ["ONI_CPHI_GB"] = str(a.cphi_gb)

    import torch
    from oni_ml_amd.config import RunConfig
    from oni_ml_amd.models.lda.settings import LDASettings
    from oni_ml_amd.pipeline import flow as P
    from oni_ml_amd.synth.flow import generate_flow_day

    def log(*x, **k):
        print(f"[{time.strftime('%H:%M:%S')}]", *x, flush=True)

    inp, lpath = os.path.join(a.workdir, "in"), os.path.join(a.workdir, "run")
    shutil.rmtree(a.workdir, ignore_errors=True)
    os.makedirs(lpath)
    t0 = time.perf_counter()
    gen = generate_flow_day(inp + "/", events=a.events, seed=5, chunk_events=-(-a.events // a.days), threads=a.threads)
    gen_s = time.perf_counter() - t0
    in_bytes = sum(os.path.getsize(p) for p in gen["paths"])
    log(f"generated {a.events} events in {len(gen['paths'])} files ({in_bytes / 1e9:.2f} GB, {gen['ips']} addresses)"
        f" in {gen_s:.1f}s")

    st = LDASettings(em_max_iter=a.em_iters)
    st.gs_updates = a.gs_updates
    st.lag = a.lag          # each %03d save of a 6M-document gamma is ~8 GB of text
    cfg = RunConfig(fdate="20160122", dsource="flow", lpath=lpath, flow_path=inp, topics=a.topics, backend=a.backend,
                    threads=a.threads, write_doc_wc=False, verbose=True, settings=st,
                    compat="strict" if a.topics == 20 else "fixed")
    cfg.validate()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if dev.type == "cuda":
        torch.cuda.reset_peak_memory_stats()
    t1 = time.perf_counter()
    summary = P.run(cfg, device=dev, log=log)
    wall = time.perf_counter() - t1
    stages = summary.get("stage_seconds", {})
    lda = {}
    mpath = os.path.join(lpath, "lda_stats.json")
    if os.path.exists(mpath):
        with open(mpath) as f:
            lda = json.load(f)
    m = lda.get("metrics", {})
    em_it = summary.get("lda", {}).get("em_iterations") or 0
    rec = dict(config="BASELINE config 5: netflow month, K=%d, fp64 block Gauss-Seidel" % a.topics,
               events=a.events, part_files=len(gen["paths"]), input_gb=round(in_bytes / 1e9, 3), addresses=gen["ips"],
               generate_s=round(gen_s, 2), corpus=summary.get("corpus"), stage_seconds=stages,
               pipeline_wall_s=round(wall, 2), em_iterations=em_it,
               lda_seconds=summary.get("lda", {}).get("seconds"), lda_timing=summary.get("lda", {}).get("timing"),
               ms_per_em_iteration=(round(1e3 * summary["lda"]["seconds"] / em_it, 2) if em_it else None),
               ingest_mb_per_s=round(in_bytes / 1e6 / stages["load"], 1) if stages.get("load") else None,
               flagged=summary.get("scored"), lda_metrics={k: v for k, v in m.items() if not isinstance(v, list)},
               peak_hbm_gb=(round(torch.cuda.max_memory_allocated() / 2**30, 2) if dev.type == "cuda" else None),
               device=(torch.cuda.get_device_name(0) if dev.type == "cuda" else "cpu"), backend=a.backend,
               threads=a.threads, lag=a.lag, cphi_gb=a.cphi_gb, gs_updates=a.gs_updates, output_gb=round(_du(lpath) / 1e9, 3), data="synthetic (synth/flow.py, scaled address pool)")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1, default=str)
    log(json.dumps(rec, default=str))
    if not a.keep:
        shutil.rmtree(a.workdir, ignore_errors=True)


if __name__ == "__main__":
    main()
