#!/usr/bin/env python
"""Per-kernel PMC counter table from a rocprofv3 --pmc database (counters_collection view).

  python scripts/pmc_summary.py results.db [--match gs_] [--md out.md]
Sums each counter over the dispatches of a kernel and prints one row per kernel, with derived
VALU instructions per wave and per busy cycle where the inputs are present."""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for name, cnt, val, did, dur in c.execute(
            "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
        if a.match not in name:
            continue
        short = name.split("(")[0][:60]
        agg[short][cnt] += float(val)
        disp[short].add((did, dur))
    cols = sorted({k for v in agg.values() for k in v})
    lines = ["| kernel | dispatches | mean us | " + " | ".join(cols) + " | VALU/wave |",
             "|---" * (len(cols) + 4) + "|"]
    for k, v in agg.items():
        d = disp[k]
        mean_us = sum(x[1] for x in d) / max(len(d), 1) / 1e3
        vw = v.get("SQ_INSTS_VALU", 0) / v["SQ_WAVES"] if v.get("SQ_WAVES") else float("nan")
        lines.append(f"| `{k}` | {len(d)} | {mean_us:.1f} | " + " | ".join(f"{v[c]:.4g}" for c in cols) +
                     f" | {vw:.1f} |")
    out = "\n".join(lines)
    print(out)
    if a.md:
        open(a.md, "w").write(out + "\n")


if __name__ == "__main__":
    main()
