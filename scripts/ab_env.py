"""A/B of environment switches on the 1-GPU headline bench.

    python scripts/ab_env.py --rounds 3 ONI_GS_PAIR_REDUCE=0 ONI_GS_PAIR_REDUCE=1 -- --steps 200

Each round runs `bench.py` once per variant (interleaved, so drift hits every variant alike) as a
child process with that variable set, and prints the child's ms_per_step.
"""
import argparse
import json
import os
import subprocess
import sys


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("variants", nargs="+", help="NAME=VALUE[,NAME=VALUE...]")
    a = ap.parse_args(argv)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {v: [] for v in a.variants}
    for r in range(1, a.rounds + 1):
        for v in a.variants:
            env = dict(os.environ)
            for kv in v.split(","):
                k, _, val = kv.partition("=")
                env[k] = val
            p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + extra, env=env, cwd=root,
                               capture_output=True, text=True, timeout=a.timeout)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                sys.exit(p.returncode)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
            ms = json.loads(line)["ms_per_step"]
            res[v].append(ms)
            print(f"round {r}  {v}  ms_per_step={ms}", flush=True)
    for v, xs in res.items():
        print(f"median {v}: {sorted(xs)[len(xs) // 2]}")


if __name__ == "__main__":
    main()
