"""Length-bucket edges at K > 32, swept on the GPU: each variant patches GSPlan.EDGES in a fresh child
process and runs bench.py's EM-iteration timing (--converge 0, no e2e legs).

    python scripts/edges_sweep.py --events 12500000 100000000 --variants default t4all t8_4k
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def variants():
    from oni_ml_amd.ops import hip as H
    return {
        "default": None,
        # no 8-wave team: every document of 257+ words (not split) on 4-wave workgroups (2 per CU)
        "t4all": ((H.GS_TEAM4, 256, None), (H.GS_SMALL, None, 256)),
        # the 8-wave team only past 4,096 words
        "t8_4k": ((H.GS_TEAM8, 4096, None), (H.GS_TEAM4, 256, 4096), (H.GS_SMALL, None, 256)),
        "t8_8k": ((H.GS_TEAM8, 8192, None), (H.GS_TEAM4, 256, 8192), (H.GS_SMALL, None, 256)),
        # the 16-lane kernel (no barrier, four documents per wave) up to 512 / 1,024 words instead of 256
        "s512": ((H.GS_TEAM8, 2048, None), (H.GS_TEAM4, 512, 2048), (H.GS_SMALL, None, 512)),
        "s1024": ((H.GS_TEAM8, 2048, None), (H.GS_TEAM4, 1024, 2048), (H.GS_SMALL, None, 1024)),
        # the 16-lane kernel only up to 128 words (the 4-wave team from 129)
        "s128": ((H.GS_TEAM8, 2048, None), (H.GS_TEAM4, 128, 2048), (H.GS_SMALL, None, 128)),
    }


def child(variant, argv):
    sys.path.insert(0, ROOT)
    from oni_ml_amd.ops import hip as H
    e = variants()[variant]
    if e is not None:
        H.GSPlan.EDGES = e
    import runpy
    sys.argv = ["bench.py"] + argv
    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--events", type=int, nargs="+", default=[12500000])
    ap.add_argument("--variants", nargs="+", default=["default", "t4all", "t8_4k"])
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--timeout", type=float, default=400)
    if len(sys.argv) > 2 and sys.argv[1] == "--child":   # child: bench.py's own arguments follow the variant
        child(sys.argv[2], sys.argv[3:])
        return 0
    a = ap.parse_args()
    for ev in a.events:
        for v in a.variants:
            argv = ["--topics", "100", "--events", str(ev), "--steps", str(a.steps), "--warmup", "2",
                    "--converge", "0", "--e2e", "0", "--e2e-cold", "0"]
            try:
                r = subprocess.run([sys.executable, "-u", __file__, "--child", v] + argv, capture_output=True,
                                   text=True, timeout=a.timeout)
            except subprocess.TimeoutExpired:
                print(json.dumps(dict(events=ev, variant=v, error="timeout")), flush=True)
                return 1
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not line:
                print(json.dumps(dict(events=ev, variant=v, rc=r.returncode, err=r.stderr[-1500:])), flush=True)
                return 1
            d = json.loads(line[-1])
            print(json.dumps(dict(events=ev, variant=v, ms=d["ms_per_step"])), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
