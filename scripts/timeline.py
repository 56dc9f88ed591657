#!/usr/bin/env python
"""Kernel timeline of a rocprofv3 trace: per-dispatch start/end relative to the first kernel of a
window, plus concurrency (how many kernels overlap) -- to check the multi-stream E-step overlap.

  python scripts/timeline.py results.db [--match lda_] [--last-ms 3]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-ms", type=float, default=2.0, help="window: the last N ms of kernels")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = [(n, s, e) for n, s, e in c.execute(f"select {name}, start, end from kernels order by start")]
    if not rows:
        return
    tend = max(e for _, _, e in rows)
    t0 = tend - a.last_ms * 1e6
    win = [(n, s, e) for n, s, e in rows if s >= t0 and a.match in n]
    base = min(s for _, s, _ in win)
    for n, s, e in win:
        short = n.split("(")[0].replace("void ", "")[-60:]
        print(f"{(s - base) / 1e3:9.1f} {(e - base) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {short}")
    # busy time (union of intervals) vs sum of durations
    iv = sorted((s, e) for _, s, e in win)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    tot = sum(e - s for s, e in iv)
    print(f"window {(max(e for _, e in iv) - base) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"sum of kernel times {tot / 1e3:.1f} us, mean concurrency {tot / max(busy, 1):.2f}")


if __name__ == "__main__":
    main()
