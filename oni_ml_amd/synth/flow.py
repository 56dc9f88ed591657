"""Synthetic netflow day in the reference's 27-column CSV schema (README.md:42-70,
flow_pre_lda.scala:46-72), calibrated on the sample cuts in the reference's
`flow_qtiles` file (ibyt deciles 0..1.8e9, ipkt up to 7.7e6, hour-of-day
deciles 0..23.98).

Shape of the data (SURVEY.md §7.2 phase 0):
* IP popularity is Zipfian over an internal /16 and an external address pool,
  so per-IP documents are heavy-tailed (a few servers / gateways see most flows);
* the port mix covers all four adjust_port cases (one side <= 1024, both
  ephemeral, one side zero, both zero / both well-known);
* a diurnal hour-of-day profile; byte and packet counts log-normal with a
  heavy upper tail.

Writing goes through the C++ formatter, so a 1M-row day takes about a second.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from ..ops import native

HEADER = ("time,year,month,day,hour,minute,second,tdur,sip,dip,sport,dport,proto,flag,fwd,stos,"
          "ipkt,ibyt,opkt,obyt,input,output,sas,das,dtos,dir,rip")

WELL_KNOWN = np.array([80, 443, 53, 22, 25, 123, 110, 143, 389, 445, 993, 995, 161, 514, 21, 23, 135, 137, 139,
                       636, 873, 1024, 8], np.int64)
WK_P = np.array([30, 30, 14, 4, 3, 3, 1, 1, 1.5, 2, 1, 1, 1, 0.5, 0.5, 0.3, 0.5, 0.5, 0.5, 0.3, 0.2, 0.2, 0.2])


def _ip_names(n_int: int, n_ext: int, rng) -> list:
    names = []
    for i in range(n_int):
        names.append(f"10.{(i >> 16) & 255}.{(i >> 8) & 255}.{i & 255}")
    ext = rng.choice(2**32 - 2**24, size=n_ext, replace=False) + 2**24
    for v in ext.tolist():
        names.append(f"{(v >> 24) & 255}.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}")
    return names


def ip_population(events: int):
    """(internal, external) address pool sizes: 40k / 120k up to 1M events (the bench day), then
    growing as events^0.8, so a 100M-event month holds a few million documents (BASELINE config 5)."""
    if events <= 1_000_000:
        return 40_000, 120_000
    f = (events / 1_000_000) ** 0.8
    return int(40_000 * f), int(120_000 * f)


def generate_flow_day(path: str, events: int = 1_000_000, seed: int = 0, date=(2016, 1, 22),
                      n_internal: Optional[int] = None, n_external: Optional[int] = None, files: int = 1,
                      threads: int = 8, chunk_events: int = 0) -> dict:
    """Write `files` CSV part files (each with the header line) under `path` (a directory) or to `path`.

    The address pool scales with `events` (ip_population) unless given.  chunk_events > 0: generate
    and write part file by part file (files = ceil(events / chunk_events)), each from its own random
    stream, so a 100M-event month never holds more than one chunk's columns in memory.
    Returns dict(paths=[...], events=n, ips=#distinct names).
    """
    di, de = ip_population(events)
    n_internal = di if n_internal is None else n_internal
    n_external = de if n_external is None else n_external
    if chunk_events and events > chunk_events:
        return _generate_chunked(path, events, seed, date, n_internal, n_external, threads, chunk_events)
    rng = np.random.default_rng(seed)
    N = native.lib()
    ips = _ip_names(n_internal, n_external, rng)
    nip = len(ips)
    # Zipf popularity over a random permutation of the pool
    pop = 1.0 / np.arange(1, nip + 1) ** 1.05
    pop /= pop.sum()
    perm = rng.permutation(nip)
    return _write_events(path, events, rng, ips, pop, perm, date, files, threads, N)


def _generate_chunked(path, events, seed, date, n_internal, n_external, threads, chunk):
    rng0 = np.random.default_rng(seed)
    N = native.lib()
    ips = _ip_names(n_internal, n_external, rng0)
    nip = len(ips)
    pop = 1.0 / np.arange(1, nip + 1) ** 1.05
    pop /= pop.sum()
    perm = rng0.permutation(nip)
    os.makedirs(path, exist_ok=True)
    nfiles = -(-events // chunk)
    paths = []
    for i in range(nfiles):
        n = min(chunk, events - i * chunk)
        rng = np.random.default_rng([seed, i + 1])
        p = os.path.join(path, f"part-{i:05d}.csv")
        _write_events(p, n, rng, ips, pop, perm, date, 1, threads, N)
        paths.append(p)
    return dict(paths=paths, events=events, ips=nip)


def _write_events(path, events, rng, ips, pop, perm, date, files, threads, N) -> dict:
    nip = len(ips)
    sip = perm[rng.choice(nip, size=events, p=pop)].astype(np.int32)
    dip = perm[rng.choice(nip, size=events, p=pop)].astype(np.int32)
    same = sip == dip
    dip[same] = (dip[same] + 1) % nip
    # ports: mixture of cases
    u = rng.random(events)
    wk = rng.choice(WELL_KNOWN, size=events, p=WK_P / WK_P.sum())
    eph = rng.integers(1025, 65536, size=events)
    eph2 = rng.integers(1025, 65536, size=events)
    sport = np.where(u < 0.45, eph, wk)                       # client -> server
    dport = np.where(u < 0.45, wk, eph)                       # server -> client
    c3 = (u >= 0.80) & (u < 0.92)                             # both ephemeral (p2p)
    sport = np.where(c3, eph, sport)
    dport = np.where(c3, eph2, dport)
    c4 = (u >= 0.92) & (u < 0.97)                             # one side zero (ICMP-ish)
    z = rng.random(events) < 0.5
    sport = np.where(c4 & z, 0, sport)
    dport = np.where(c4 & ~z, 0, dport)
    c1 = u >= 0.97                                            # both well-known / both zero
    sport = np.where(c1, rng.choice(WELL_KNOWN, size=events), sport)
    dport = np.where(c1, np.where(rng.random(events) < 0.3, 0, rng.choice(WELL_KNOWN, size=events)), dport)
    proto_id = np.where(c4, 2, np.where(rng.random(events) < 0.8, 0, 1)).astype(np.int32)
    # time of day: diurnal mixture
    hour_p = 0.4 + np.sin((np.arange(24) - 6) / 24 * 2 * np.pi).clip(-0.6, 1.0) + 0.6
    hour_p /= hour_p.sum()
    hour = rng.choice(24, size=events, p=hour_p)
    minute = rng.integers(0, 60, size=events)
    second = rng.integers(0, 60, size=events)
    order = np.lexsort((second, minute, hour))
    hour, minute, second = hour[order], minute[order], second[order]
    sip, dip, sport, dport, proto_id = sip[order], dip[order], sport[order], dport[order], proto_id[order]
    # packets/bytes (calibrated to flow_qtiles: median pkt ~1-2, bytes deciles 52..3569, heavy tail)
    ipkt = np.maximum(1, np.round(np.exp(rng.normal(0.35, 1.15, size=events)))).astype(np.int64)
    big = rng.random(events) < 0.002
    ipkt[big] *= rng.integers(100, 5000, size=int(big.sum()))
    per = np.exp(rng.normal(4.6, 0.9, size=events))
    ibyt = np.maximum(28, np.round(ipkt * per)).astype(np.int64)
    opkt = (ipkt * rng.random(events) * 1.2).astype(np.int64)
    obyt = (opkt * per * rng.random(events)).astype(np.int64)
    tdur = np.round(rng.exponential(2.0, size=events) * (ipkt > 1), 3)
    y, mo, d = date
    sod = (hour * 3600 + minute * 60 + second).astype(np.int32)
    tnames = [f"{y:04d}-{mo:02d}-{d:02d} {h:02d}:{m:02d}:{s:02d}" for h in range(24) for m in range(60) for s in range(60)]
    flags = [".A....", ".AP.SF", "...R..", ".A..S.", "......", ".AP..."]
    flag_id = rng.integers(0, len(flags), size=events).astype(np.int32)
    rip_names = ["10.219.32.250", "10.219.32.251"]
    rip_id = rng.integers(0, 2, size=events).astype(np.int32)
    zeros = np.zeros(events, np.int64)
    in_if = rng.integers(0, 12, size=events)
    out_if = rng.integers(0, 12, size=events)
    cols = [
        ("dict", tnames, sod), ("const", str(y)), ("const", str(mo)), ("const", str(d)),
        ("int", hour.astype(np.int64)), ("int", minute.astype(np.int64)), ("int", second.astype(np.int64)),
        ("java", tdur.astype(np.float64)),
        ("dict", ips, sip), ("dict", ips, dip),
        ("int", sport.astype(np.int64)), ("int", dport.astype(np.int64)),
        ("dict", ["TCP", "UDP", "ICMP"], proto_id), ("dict", flags, flag_id),
        ("int", zeros), ("int", zeros), ("int", ipkt), ("int", ibyt), ("int", opkt), ("int", obyt),
        ("int", in_if.astype(np.int64)), ("int", out_if.astype(np.int64)), ("int", zeros), ("int", zeros),
        ("int", zeros), ("int", zeros), ("dict", rip_names, rip_id),
    ]
    if files > 1 or os.path.isdir(path) or path.endswith("/"):
        os.makedirs(path, exist_ok=True)
        paths = [os.path.join(path, f"part-{i:05d}.csv") for i in range(files)]
    else:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        paths = [path]
    bounds = np.linspace(0, events, len(paths) + 1).astype(np.int64)
    for i, p in enumerate(paths):
        with open(p, "w") as f:
            f.write(HEADER + "\n")
        order_i = np.arange(bounds[i], bounds[i + 1], dtype=np.int64)
        N.write_rows(p, order_i, cols, append=True, threads=threads)
    return dict(paths=paths, events=events, ips=nip)


def generate_flow_feedback(path: str, table_rows: list, seed: int = 0, n: int = 20) -> int:
    """Write a flow_scores.csv (22 columns + header, flow_pre_lda.scala:150-171) marking `n` events
    of `table_rows` (list of 27-field CSV lines) with severity 3 (non-threatening) and a few others."""
    rng = np.random.default_rng(seed)
    hdr = ("sev,tstart,srcIP,dstIP,sport,dport,proto,flag,ipkt,ibyt,lda_score,rank,srcIpInternal,destIpInternal,"
           "srcGeo,dstGeo,srcDomain,dstDomain,gtiSrcRep,gtiDstRep,norseSrcRep,norseDstRep")
    pick = rng.choice(len(table_rows), size=min(len(table_rows), 2 * n), replace=False)
    lines = [hdr]
    for j, i in enumerate(pick.tolist()):
        f = table_rows[i].split(",")
        sev = 3 if j < n else int(rng.integers(1, 3))
        row = [str(sev), f[0], f[8], f[9], f[10], f[11], f[12], f[13], f[16], f[17], "1e-21", str(j), "1", "0",
               "US", "US", "-", "-", "-", "-", "-", "-"]
        lines.append(",".join(row))
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    return n
