"""DNS input ingest without torch: the selected parquet columns with the reference's row rules, the
analyst feedback rows and the top-1m list (dns_pre_lda.scala:62-66,84-148).  Kept free of torch so
`ml_ops` can read the day's parquet on a thread while the interpreter is still importing torch
(`pipeline/prefetch.py`); `features/dns.py` re-exports every name."""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from ..ops import native

COLUMNS = ["frame_time", "unix_tstamp", "frame_len", "ip_dst", "dns_qry_name", "dns_qry_class", "dns_qry_type",
           "dns_qry_rcode"]
FEEDBACK_IDX = dict(frame_time=0, unix_tstamp=23, frame_len=1, ip_dst=2, dns_qry_name=3, dns_qry_class=4,
                    dns_qry_type=5, dns_qry_rcode=6, dns_sev=18)


_ARROW_THREADS = False


def _pa():
    global _ARROW_THREADS
    import pyarrow as pa
    import pyarrow.compute as pc
    import pyarrow.parquet as pq
    if not _ARROW_THREADS:
        # Arrow sizes its pool by the machine's cores (hundreds on a GPU host, of which a job gets 16):
        # cap it at this process's share so a parquet read beside the torch import does not swamp it
        _ARROW_THREADS = True
        try:
            n = (int(os.environ.get("ONI_THREADS") or 0) or int(os.environ.get("OMP_NUM_THREADS") or 0)
                 or min(os.cpu_count() or 8, 16))
            if pa.cpu_count() > n:
                pa.set_cpu_count(n)
        except (ValueError, AttributeError):
            pass
    return pa, pc, pq


def select_paths(dns_path: str, strict: bool) -> List[str]:
    paths = [p for p in dns_path.split(",")]
    if strict:
        return [p for i, p in enumerate(paths) if i == 0 or i > 1]
    return [p for p in paths if p]


def _java_split_len(line: str) -> int:
    parts = line.split(",")
    while parts and parts[-1] == "":
        parts.pop()
    return len(parts) if line else 1


def read_dns_feedback(path: str) -> List[List[str]]:
    """dns_scores.csv rows with dns_sev == 3 as the 8 selected string fields."""
    if not path or not os.path.exists(path):
        return []
    with open(path, "r", encoding="utf-8", newline="") as fh:
        lines = fh.read().split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    out = []
    for l in lines[1:]:
        f = l.rstrip("\r").split(",")
        while f and f[-1] == "":
            f.pop()
        if len(f) < 24:
            continue   # the reference would throw ArrayIndexOutOfBounds
        try:
            flen = int(f[FEEDBACK_IDX["frame_len"]].strip())
            sev = int(f[FEEDBACK_IDX["dns_sev"]].strip())
        except ValueError:
            continue
        if sev != 3:
            continue
        row = [f[FEEDBACK_IDX[c]] for c in COLUMNS]
        row[2] = str(flen)
        out.append(row)
    return out


def _java_double(s: str) -> Optional[float]:
    return native.lib().java_parse_double(s)


@dataclass
class DnsTable:
    """The 8 selected columns as strings (mkString semantics) + weights; feedback rows last.

    Columns stay Arrow string arrays (one chunk each): featurization reads the name bytes and
    offsets zero-copy and dictionary-encodes with Arrow kernels; only the flagged output rows are
    ever turned into Python strings (``take``)."""
    arrays: Dict[str, object]      # name -> pyarrow StringArray over all n rows
    frame_len: np.ndarray          # f64
    unix_tstamp: np.ndarray        # f64
    weight: np.ndarray             # int64
    n_raw: int
    n_feedback: int
    dropped: int = 0

    @property
    def n(self) -> int:
        return self.n_raw + self.n_feedback

    def column(self, name: str, n: Optional[int] = None):
        a = self.arrays[name]
        return a if n is None or n == len(a) else a.slice(0, n)

    def take(self, name: str, rows) -> List[str]:
        pa, pc, _ = _pa()
        return pc.take(self.arrays[name], pa.array(np.asarray(rows, np.int64))).to_pylist()

    def take_encoded(self, name: str, rows):
        """(first-appearance ids int32, distinct names) of column ``name`` at ``rows`` -- what
        ``dictionary_encode(take(...))`` returns, from Arrow's dictionary encoding (indices in order of
        first occurrence): only the distinct names become Python strings (a cold DNS day flags 505 k
        queries x 8 columns: 1.6 s of Python lists and dict probes before)."""
        pa, pc, _ = _pa()
        t = pc.take(self.arrays[name], pa.array(np.asarray(rows, np.int64)))
        if isinstance(t, pa.ChunkedArray):
            t = t.combine_chunks()
        d = pc.dictionary_encode(t)
        return np.asarray(d.indices.to_numpy(zero_copy_only=False), np.int32), d.dictionary.to_pylist()

    @property
    def cols(self) -> Dict[str, list]:
        """All columns as Python lists (tests / small tables only)."""
        return {c: a.to_pylist() for c, a in self.arrays.items()}


def _arrow_strings(pa, pc, col):
    if not pa.types.is_string(col.type) and not pa.types.is_large_string(col.type):
        col = pc.cast(col, pa.string())
    return pc.fill_null(col, "null")


def load_dns(dns_path: str, feedback_path: Optional[str] = None, dupfactor: int = 1000, strict: bool = True) -> DnsTable:
    pa, pc, pq = _pa()
    tables = []
    for p in select_paths(dns_path, strict):
        if not p:
            continue
        # a single file through ParquetFile: pq.read_table would import the dataset layer (0.1 s cold)
        tables.append(pq.ParquetFile(p).read(columns=COLUMNS) if os.path.isfile(p) else pq.read_table(p, columns=COLUMNS))
    if not tables:
        raise FileNotFoundError(f"no DNS input in {dns_path!r}")
    fb = read_dns_feedback(feedback_path) if feedback_path else []
    return table_from_arrow(tables, fb, dupfactor)


def _parquet_files(p: str) -> List[str]:
    """The files pq.read_table reads for ``p`` (a file, or a directory dataset), in its order."""
    if os.path.isdir(p):
        import pyarrow.dataset as ds
        return list(ds.dataset(p, format="parquet").files)
    return [p]


def load_dns_rows(dns_path: str, lo: int, hi: int, strict: bool = True):
    """Rows [lo, hi) of the selected parquet inputs taken as one table (before the null filter): only
    the row groups holding them are read (the row-sharded DNS ingest, pipeline/sharded.py)."""
    pa, pc, pq = _pa()
    out, off = [], 0
    for p in [f for q in select_paths(dns_path, strict) if q for f in _parquet_files(q)]:
        f = pq.ParquetFile(p)
        for g in range(f.metadata.num_row_groups):
            n = f.metadata.row_group(g).num_rows
            a, b = max(lo, off), min(hi, off + n)
            if a < b:
                t = f.read_row_group(g, columns=COLUMNS)
                out.append(t.slice(a - off, b - a))
            off += n
    return out


def dns_total_rows(dns_path: str, strict: bool = True) -> int:
    _, _, pq = _pa()
    return sum(pq.ParquetFile(f).metadata.num_rows for p in select_paths(dns_path, strict) if p
               for f in _parquet_files(p))


def table_from_arrow(tables, fb, dupfactor: int = 1000) -> DnsTable:
    """The reference's row rules on the read tables (in order) + the feedback rows (weight DUPFACTOR)."""
    pa, pc, pq = _pa()
    tables = [t.filter(pc.and_(pc.is_valid(t["frame_len"]), pc.is_valid(t["unix_tstamp"]))) for t in tables]
    if not tables:
        t = pa.table({c: pa.array([], pa.string()) for c in COLUMNS})
    else:
        t = pa.concat_tables(tables, promote_options="permissive") if len(tables) > 1 else tables[0]
    strs = {c: _arrow_strings(pa, pc, t[c]).combine_chunks() for c in COLUMNS}
    # Row.mkString(",").split(",") must give back 8 fields: no comma anywhere; trailing empty fields vanish
    bad = None
    for c in COLUMNS:
        m = pc.match_substring(strs[c], ",")
        bad = m if bad is None else pc.or_(bad, m)
    bad = pc.or_(bad, pc.equal(pc.utf8_length(strs[COLUMNS[-1]]), 0))
    keep = pc.invert(bad)
    n_before = len(t)
    strs = {c: pc.filter(v, keep) for c, v in strs.items()}
    if len(t):
        flen = pc.filter(t["frame_len"], keep).to_numpy(zero_copy_only=False).astype(np.float64)
        tst = pc.filter(t["unix_tstamp"], keep).to_numpy(zero_copy_only=False).astype(np.float64)
    else:
        flen = tst = np.zeros(0, np.float64)
    n_raw = len(flen)
    fb_ok = []
    for r in fb:
        if any("," in x for x in r) or r[-1] == "":
            continue
        a, b = _java_double(r[2]), _java_double(r[1])
        if a is None or b is None:
            continue
        fb_ok.append((r, a, b))
    arrays = {}
    for j, c in enumerate(COLUMNS):
        a = strs[c]
        if fb_ok:
            a = pa.concat_arrays([a.cast(pa.large_string()), pa.array([r[j] for r, _, _ in fb_ok], pa.large_string())])
        arrays[c] = a.combine_chunks() if hasattr(a, "combine_chunks") else a
    if fb_ok:
        flen = np.concatenate([flen, np.array([a for _, a, _ in fb_ok])])
        tst = np.concatenate([tst, np.array([b for _, _, b in fb_ok])])
    w = np.ones(len(flen), np.int64)
    w[n_raw:] = dupfactor
    return DnsTable(arrays, flen, tst, w, n_raw, len(fb_ok), dropped=n_before - n_raw)


def load_top_domains(path: Optional[str]) -> List[str]:
    """top-1m.csv (`rank,domain`) -> first label of each domain (dns_pre_lda.scala:62-66)."""
    if not path or not os.path.exists(path):
        return []
    out = []
    with open(path, "r", encoding="utf-8", errors="replace") as f:
        for line in f:
            parts = line.rstrip("\n").split(",")
            if len(parts) < 2:
                continue
            out.append(parts[1].split(".")[0])
    return out


def _offsets(names):
    """(bytes buffer, int64 offsets) of a list of str or an Arrow string array (zero-copy data)."""
    if isinstance(names, list):
        enc = [s.encode("utf-8") for s in names]
        off = np.zeros(len(enc) + 1, np.int64)
        np.cumsum([len(b) for b in enc], out=off[1:])
        return b"".join(enc), off
    pa, _, _ = _pa()
    a = names
    wide = pa.types.is_large_string(a.type)
    bufs = a.buffers()
    off = np.frombuffer(bufs[1], dtype=np.int64 if wide else np.int32)[a.offset: a.offset + len(a) + 1]
    data = bufs[2] if bufs[2] is not None else b""
    return data, off.astype(np.int64)


def arrow_dictionary_encode(arr):
    """First-appearance ids + names of an Arrow string array (Arrow's hash memo assigns codes in
    order of first occurrence, like ``dictionary_encode``)."""
    _, pc, _ = _pa()
    d = pc.dictionary_encode(arr)
    return d.indices.to_numpy(zero_copy_only=False).astype(np.int32), d.dictionary.to_pylist()


def host_features(tab: DnsTable, top_domains, threads: int = 8, n: Optional[int] = None, cuts: bool = False) -> dict:
    """The torch-free part of dns_pre over every row of ``tab``: the C++ name features (domain, subdomain,
    lengths, entropy, top-1m flag), and the first-appearance dictionaries of "qry_type_qry_rcode" and of
    ip_dst.  `pipeline/prefetch.py` runs it on the input thread while torch imports; features/dns.py's
    ``featurize`` takes it (``host``) for the whole table or any prefix of it (the raw rows: a prefix of a
    first-appearance encoding is the encoding of the prefix)."""
    from .dns_data import COUNTRY_CODES, SPECIAL_DOMAIN
    pa, pc, _ = _pa()
    n = tab.n if n is None else n
    data, off = _offsets(tab.column("dns_qry_name", n))
    F = native.lib().dns_features(data, off, list(COUNTRY_CODES), list(top_domains), SPECIAL_DOMAIN, threads)
    qt, qr = tab.column("dns_qry_type", n), tab.column("dns_qry_rcode", n)
    # the separator must have the columns' type (large_string once feedback rows are appended)
    F["_qid"], F["_qnames"] = arrow_dictionary_encode(pc.binary_join_element_wise(qt, qr, pa.scalar("_", qt.type)))
    F["_ip_ids"], F["_ip_names"] = arrow_dictionary_encode(tab.column("ip_dst", n))
    if cuts:
        # dns_pre's cuts (every row) and dns_post's (the raw rows: the reference recomputes them there)
        from .cuts_host import dns_cuts_np
        vals = dict(unix_tstamp=tab.unix_tstamp, frame_len=tab.frame_len, subdomain_length=F["subdomain_length"],
                    entropy=F["entropy"], num_periods=F["num_periods"])
        F["_cuts"] = {m: dns_cuts_np(vals, tab.weight, m, threads) for m in sorted({n, min(n, tab.n_raw)})}
    return F

