#!/usr/bin/env python
"""Per-rank stage times of the row-sharded ``ml_ops`` pipeline (pipeline/sharded.py).

Generates one synthetic day, then runs ``oni_ml_amd.cli ml_ops YYYYMMDD <flow|dns> TOL`` with
N = 1, 2, 4 ... ranks (torchrun; several ranks on one GPU rehearse over gloo -- ONI_DIST_BACKEND
=gloo -- exactly as the 8-GPU RCCL run splits the work) and reads every rank's metrics file
(metrics.jsonl / metrics.rank<r>.jsonl).  Reports, per N, the pipeline wall, each stage's seconds
on every rank, and rank 0's serial share: the seconds rank 0 spends in stages beyond the slowest
other rank, over the wall.

  python scripts/pipeline_ranks.py --events 1000000 --ranks 1,4 --md out.md --json out.json
  BASELINE config 5 (a month, K = 100) on 8 ranks sharing one GPU, a TOL that flags events:
  python scripts/pipeline_ranks.py --events 100000000 --days 30 --topics 100 --compat fixed --tol 1e-9 --ranks 8
"""
import argparse
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STAGES = {"flow": ["load", "flow_pre", "lda_pre", "lda", "lda_post", "flow_post"],
          "dns": ["load", "dns_pre", "lda_pre", "lda", "lda_post", "dns_post"]}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--source", default="flow", choices=["flow", "dns"])
    ap.add_argument("--events", type=int, default=1_000_000)
    ap.add_argument("--ranks", default="1,4")
    ap.add_argument("--tol", default=None)
    ap.add_argument("--backend", default="gloo", help="collective backend of the ranks (gloo: many ranks per GPU)")
    ap.add_argument("--lda-backend", default="auto")
    ap.add_argument("--md")
    ap.add_argument("--json")
    ap.add_argument("--timeout", type=int, default=900)
    ap.add_argument("--days", type=int, default=1, help="flow: part files (one per day) of the generated input")
    ap.add_argument("--topics", type=int, default=20)
    ap.add_argument("--compat", default=None, help="strict | fixed (default: strict at K = 20, else fixed)")
    ap.add_argument("--threads", type=int, default=8, help="native threads per rank (0: no --threads, the "
                                                               "rank's CPU budget decides, utils/hostres.py)")
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE set for the ml_ops processes")
    ap.add_argument("--variants", default="", help="';'-separated env variants (KEY=VAL,KEY=VAL) run back to back "
                                                   "at every N on the same input (e.g. 'ONI_THREADS=16;')")
    ap.add_argument("--split-threads", action="store_true", help="--threads is the box's share: N ranks get threads / N each")
    ap.add_argument("--cphi-gb", default=None, help="per-rank HBM budget of the c.phi rows")
    ap.add_argument("--no-word-assignments", action="store_true")
    ap.add_argument("--lag", default=None, help="LAG save period (lda-c: 5; 0: only 000 and final)")
    ap.add_argument("--tol-quantile", type=float, default=None,
                    help="calibrate TOL: a first run at --tol records the score quantiles, every listed N then runs "
                         "at its key_q<Q> (so about Q of the events are flagged); Q in 1e-4, 1e-3, 1e-2, 0.1")
    ap.add_argument("--cprofile", default=None, help="one-process runs under cProfile, stats written here")
    a = ap.parse_args()
    t_start = time.perf_counter()

    def heartbeat():     # a long generation / config-5 run prints nothing for minutes otherwise
        while True:
            time.sleep(60)
            print(json.dumps(dict(heartbeat_s=round(time.perf_counter() - t_start))), flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    tol = a.tol or ("1e-5" if a.source == "flow" else "1e-4")
    tmp = tempfile.mkdtemp(prefix="oni_ranks_")
    out = dict(source=a.source, events=a.events, backend=a.backend, runs=[])
    try:
        if a.source == "flow":
            from oni_ml_amd.synth.flow import generate_flow_day
            tg = time.perf_counter()
            generate_flow_day(os.path.join(tmp, "in/"), events=a.events, seed=7,
                              chunk_events=-(-a.events // a.days) if a.days > 1 else 0, threads=16)
            out["generate_s"] = round(time.perf_counter() - tg, 2)
            print(json.dumps(dict(generated=a.events, seconds=out["generate_s"])), flush=True)
            inp = ["--flow-path", os.path.join(tmp, "in")]
        else:
            from oni_ml_amd.synth.dns import generate_dns_day
            g = generate_dns_day(os.path.join(tmp, "in"), events=a.events, seed=7, files=4,
                                 n_names=max(20_000, a.events // 10), n_clients=max(5_000, a.events // 40),
                                 with_edge_rows=False)
            inp = ["--dns-path", g["dns_path"], "--top1m", g["top1m"]]
        ns = [int(x) for x in a.ranks.split(",")]
        variants = a.variants.split(";") if a.variants else [""]
        plan = ([("calibration", ns[0], "")] if a.tol_quantile else []) + [("run", n, v) for n in ns for v in variants]
        for kind, n, variant in plan:
            lp = os.path.join(tmp, f"ml{n}")
            compat = a.compat or ("strict" if a.topics == 20 else "fixed")
            cli = ["-m", "oni_ml_amd", "ml_ops", "20160122", a.source, tol, "--lpath", lp, "--gpus", str(n),
                   "--conf", "/nonexistent", "--quiet", "--backend", a.lda_backend, "--topics", str(a.topics),
                   "--compat", compat] + (["--threads", str(max(1, a.threads // n) if a.split_threads else a.threads)]
                                          if a.threads > 0 else []) + inp
            if a.cphi_gb:
                cli += ["--cphi-gb", str(a.cphi_gb)]
            if a.no_word_assignments:
                cli += ["--no-word-assignments"]
            if a.lag is not None:
                cli += ["--lag", str(a.lag)]
            if a.cprofile and n == 1:    # the whole one-process run under cProfile (no fast exit: it writes at exit)
                cli = ["-m", "cProfile", "-o", a.cprofile] + cli
            cmd = [sys.executable] + (cli if n == 1 else
                                      ["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                                       "--master-addr", "127.0.0.1", "--master-port", str(_port())] + cli)
            env = dict(os.environ, ONI_DIST_BACKEND=a.backend)
            env.update(dict(kv.split("=", 1) for kv in a.env))
            env.update(dict(kv.split("=", 1) for kv in variant.split(",") if kv))
            if a.cprofile:
                env["ONI_FAST_EXIT"] = "0"
            t0 = time.perf_counter()
            r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=a.timeout)
            if a.json:      # the children's stderr (e.g. ONI_PROFILE=table writer timings) next to the record
                with open(os.path.splitext(a.json)[0] + f".{kind}.N{n}.stderr.txt", "w") as fh:
                    fh.write(r.stderr[-200000:])
            wall = time.perf_counter() - t0
            if r.returncode != 0:
                print(r.stdout[-3000:], r.stderr[-6000:], file=sys.stderr)
                raise SystemExit(f"N={n} failed rc={r.returncode}")
            summ = json.load(open(os.path.join(lp, "run_summary.json")))
            per_rank = []
            for k in range(n):
                f = os.path.join(lp, "metrics.jsonl" if k == 0 else f"metrics.rank{k}.jsonl")
                st = {}
                for line in open(f):
                    rec = json.loads(line)
                    if rec.get("status") == "ok" and rec.get("stage") in STAGES[a.source]:
                        st[rec["stage"]] = st.get(rec["stage"], 0.0) + rec["seconds"]
                per_rank.append(st)
            pw = summ["wall_seconds"]
            serial = 0.0
            for s in STAGES[a.source]:
                others = [p.get(s, 0.0) for p in per_rank[1:]]
                serial += max(0.0, per_rank[0].get(s, 0.0) - (max(others) if others else 0.0))
            fp = [json.loads(l) for l in open(os.path.join(lp, "metrics.jsonl"))] if os.path.exists(
                os.path.join(lp, "metrics.jsonl")) else []
            keyq = {k: v for rec in fp if rec.get("stage") in ("flow_post", "dns_post")
                    for k, v in rec.items() if k.startswith("key_q")}
            out_gb = sum(os.path.getsize(os.path.join(d, f)) for d, _, fs in os.walk(lp) for f in fs) / 1e9
            shutil.rmtree(lp, ignore_errors=True)       # (config 5 writes ~50 GB of text per run)
            run = dict(kind=kind, variant=variant, tol=tol, ranks=n, process_wall_s=round(wall, 3), pipeline_wall_s=round(pw, 3),
                       flagged=summ.get("scored"), rank0_key_quantiles=keyq, startup_marks=summ.get("startup_marks"), corpus=summ.get("corpus"),
                       em_iterations=summ.get("lda", {}).get("em_iterations"),
                       lda_seconds=summ.get("lda", {}).get("seconds"), lda_timing=summ.get("lda", {}).get("timing"),
                       stage_s=[{k: round(v, 3) for k, v in p.items()} for p in per_rank],
                       rank0_serial_s=round(serial, 3) if n > 1 else None,
                       rank0_serial_share=round(serial / pw, 4) if n > 1 else None, output_gb=round(out_gb, 3))
            print(json.dumps(run), flush=True)
            if kind == "calibration":
                tol = repr(float(keyq[f"key_q{a.tol_quantile:g}"]))
                out["calibration"] = run
                continue
            out["runs"].append(run)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)
    if a.md:
        lines = [f"# Per-rank stage seconds, {a.source} day of {a.events} events (collectives: {a.backend})", ""]
        for run in out["runs"]:
            lines.append(f"## N = {run['ranks']}{' [' + run['variant'] + ']' if run.get('variant') else ''}: "
                         f"pipeline wall {run['pipeline_wall_s']} s, TOL {run['tol']}, "
                         f"flagged {run['flagged']}, "
                         f"EM iterations {run['em_iterations']}"
                         + (f", rank 0 serial {run['rank0_serial_s']} s = {100 * run['rank0_serial_share']:.1f} % of the wall"
                            if run["ranks"] > 1 else ""))
            lines.append("")
            lines.append("| rank | " + " | ".join(STAGES[a.source]) + " |")
            lines.append("|---" * (len(STAGES[a.source]) + 1) + "|")
            for k, p in enumerate(run["stage_s"]):
                lines.append(f"| {k} | " + " | ".join(f"{p.get(s, 0):.3f}" for s in STAGES[a.source]) + " |")
            lines.append("")
            lines.append(f"process wall {run['process_wall_s']} s; start-up marks {run['startup_marks']}; "
                         f"corpus {run['corpus']}; output {run['output_gb']} GB; rank-0 score quantiles "
                         f"{run['rank0_key_quantiles']}")
            lines.append("")
        open(a.md, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
