"""Synthetic DNS day in the reference's Hive/parquet schema (README.md:74-87) plus a fake top-1m.csv.

Columns: frame_time STRING, unix_tstamp BIGINT, frame_len INT, ip_dst STRING,
ip_src STRING, dns_qry_name STRING, dns_qry_class STRING, dns_qry_type INT,
dns_qry_rcode INT, dns_a STRING.  Query names cover every branch of the
reference's domain parser (dns_pre_lda.scala:185-220): gTLD and ccTLD names
with and without subdomains, reverse lookups under in-addr.arpa, one- and
two-label names, the special "intel" domain, CDN-style long subdomains and
high-entropy DGA-like labels; a few rows carry nulls / commas to exercise the
row filters.
"""
from __future__ import annotations

import os

import numpy as np

POPULAR = ["google", "facebook", "youtube", "amazon", "yahoo", "wikipedia", "twitter", "microsoft", "apple",
           "netflix", "linkedin", "instagram", "bing", "reddit", "ebay", "office", "live", "akamaihd", "cloudfront",
           "github", "stackoverflow", "adobe", "dropbox", "salesforce", "zoom", "paypal", "cnn", "bbc"]
GTLD = ["com", "net", "org", "io", "info", "biz"]
CCTLD = ["uk", "de", "jp", "cn", "ru", "br", "fr", "in", "au", "it"]
SUBS = ["www", "mail", "api", "cdn", "login", "static", "img", "m", "en", "video", "s3", "edge"]


def _rand_label(rng, n, alphabet="abcdefghijklmnopqrstuvwxyz0123456789"):
    a = np.frombuffer(alphabet.encode(), dtype=np.uint8)
    return bytes(rng.choice(a, size=n)).decode()


def make_names(rng, n_unique: int):
    names = []
    for i in range(n_unique):
        u = rng.random()
        dom = POPULAR[int(rng.integers(len(POPULAR)))] if rng.random() < 0.6 else _rand_label(rng, int(rng.integers(4, 12)), "abcdefghijklmnopqrstuvwxyz")
        if u < 0.40:
            names.append(f"{SUBS[int(rng.integers(len(SUBS)))]}.{dom}.{GTLD[int(rng.integers(len(GTLD)))]}")
        elif u < 0.52:
            names.append(f"{SUBS[int(rng.integers(len(SUBS)))]}.{dom}.co.{CCTLD[int(rng.integers(len(CCTLD)))]}")
        elif u < 0.60:
            names.append(f"{dom}.{GTLD[int(rng.integers(len(GTLD)))]}")
        elif u < 0.70:
            ip = rng.integers(1, 255, size=4)
            names.append(f"{ip[0]}.{ip[1]}.{ip[2]}.{ip[3]}.in-addr.arpa")
        elif u < 0.80:
            parts = [_rand_label(rng, int(rng.integers(3, 10))) for _ in range(int(rng.integers(2, 5)))]
            names.append(".".join(parts) + f".{dom}.{GTLD[int(rng.integers(len(GTLD)))]}")
        elif u < 0.90:   # DGA-like
            names.append(f"{_rand_label(rng, int(rng.integers(12, 32)))}.{GTLD[int(rng.integers(len(GTLD)))]}")
        elif u < 0.93:
            names.append(f"{SUBS[int(rng.integers(len(SUBS)))]}.intel.com")
        elif u < 0.96:
            names.append(_rand_label(rng, int(rng.integers(3, 12)), "abcdefghijklmnopqrstuvwxyz"))
        else:
            names.append(f"{SUBS[int(rng.integers(len(SUBS)))]}.{dom}.{CCTLD[int(rng.integers(len(CCTLD)))]}")
    return names


def generate_dns_day(path: str, events: int = 100_000, seed: int = 0, files: int = 1, n_names: int = 20_000,
                     n_clients: int = 5_000, date=(2016, 1, 22), with_edge_rows: bool = True) -> dict:
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(seed)
    names = make_names(rng, n_names)
    pop = 1.0 / np.arange(1, n_names + 1) ** 1.1
    pop /= pop.sum()
    qn = rng.choice(n_names, size=events, p=pop)
    cpop = 1.0 / np.arange(1, n_clients + 1) ** 0.9
    cpop /= cpop.sum()
    cl = rng.choice(n_clients, size=events, p=cpop)
    clients = [f"10.{(i >> 8) & 255}.{i & 255}.{(i * 7) % 250 + 1}" for i in range(n_clients)]
    t0 = int(np.datetime64(f"{date[0]:04d}-{date[1]:02d}-{date[2]:02d}T00:00:00").astype("datetime64[s]").astype(np.int64))
    ts = np.sort(t0 + rng.integers(0, 86400, size=events))
    qtype = rng.choice([1, 28, 5, 12, 15, 16, 33, 2, 255], size=events, p=[.55, .18, .06, .1, .04, .03, .02, .01, .01])
    rcode = rng.choice([0, 3, 2, 5], size=events, p=[.86, .1, .03, .01])
    name_len = np.fromiter((len(x) for x in names), np.int64, count=len(names))
    flen = (60 + name_len[qn] + rng.integers(0, 200, size=events) * (rng.random(events) < 0.3)).astype(np.int32)
    import pyarrow.compute as pc
    ft = np.char.add(np.char.replace(np.datetime_as_string(ts.astype("datetime64[s]")), "T", " "), ".000000000")
    # dictionary columns: one string per distinct value, indices per event (vectorised; millions of rows)
    take = lambda vals, idx: pc.take(pa.array(vals, pa.string()), pa.array(idx.astype(np.int64)))
    cols = dict(
        frame_time=pa.array(ft, pa.string()),
        unix_tstamp=pa.array(ts.astype(np.int64), pa.int64()),
        frame_len=pa.array(flen, pa.int32()),
        ip_dst=take(clients, cl),
        ip_src=take(["10.0.0.53"], np.zeros(events, np.int64)),
        dns_qry_name=take(names, qn),
        dns_qry_class=take(["0x00000001"], np.zeros(events, np.int64)),
        dns_qry_type=pa.array(qtype.astype(np.int32), pa.int32()),
        dns_qry_rcode=pa.array(rcode.astype(np.int32), pa.int32()),
        dns_a=pa.array(["93.184.216.34"] * events, pa.string()),
    )
    if with_edge_rows and events >= 10:
        # null frame_len (dropped), comma in a name (dropped), null name ("null" query), empty name
        fl = cols["frame_len"].to_pylist()
        fl[0] = None
        cols["frame_len"] = pa.array(fl, pa.int32())
        nm = cols["dns_qry_name"].to_pylist()
        nm[1] = "bad,name.example.com"
        nm[2] = None
        nm[3] = ""
        cols["dns_qry_name"] = pa.array(nm, pa.string())
    table = pa.table(cols)
    os.makedirs(path, exist_ok=True)
    paths = []
    bounds = np.linspace(0, events, files + 1).astype(np.int64)
    for i in range(files):
        d = os.path.join(path, f"h={i:02d}")
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, "part-00000.parquet")
        pq.write_table(table.slice(bounds[i], bounds[i + 1] - bounds[i]), p)
        paths.append(d)
    top = os.path.join(path, "top-1m.csv")
    with open(top, "w") as f:
        for r, dname in enumerate(POPULAR[:20] + ["example", "intel"], start=1):
            f.write(f"{r},{dname}.com\n")
    return dict(paths=paths, dns_path=",".join(paths), top1m=top, events=events)
