#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv) per kernel.

Usage: python scripts/prof_summary.py <results.db|kernel_trace.csv> [--top N] [--md out.md]
Prints: kernel name, calls, total/mean/max microseconds and share of GPU time.
"""
import argparse
import collections
import csv
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    q = f"select {name_col}, start, end from kernels"
    for name, s, e in c.execute(q):
        yield name, (e - s) / 1e3


def rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    it = rows_from_db(a.path) if a.path.endswith(".db") else rows_from_csv(a.path)
    agg = collections.defaultdict(list)
    for n, us in it:
        agg[n].append(us)
    tot = sum(sum(v) for v in agg.values()) or 1.0
    lines = ["| kernel | calls | total us | mean us | max us | % |", "|---|---|---|---|---|---|"]
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[: a.top]:
        short = n if len(n) < 110 else n[:107] + "..."
        lines.append(f"| `{short}` | {len(v)} | {sum(v):.1f} | {sum(v)/len(v):.2f} | {max(v):.1f} | {100*sum(v)/tot:.1f} |")
    lines.append(f"\nTotal GPU kernel time: {tot:.1f} us over {sum(len(v) for v in agg.values())} dispatches")
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    sys.exit(main())
