"""Flow input ingest without torch: the 27-column CSV into the native TextTable, the analyst feedback
rows, the input file list (flow_pre_lda.scala:22-26,146-270).  Kept free of torch so `ml_ops` can
start reading the day's files on a thread while the interpreter is still importing torch
(`pipeline/prefetch.py`); `features/flow.py` re-exports every name."""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional

from ..ops import native

NCOLS = 27
C_HOUR, C_MIN, C_SEC, C_SIP, C_DIP, C_A, C_B, C_IPKT, C_IBYT = 4, 5, 6, 8, 9, 10, 11, 16, 17
NUMERIC = [C_HOUR, C_MIN, C_SEC, C_A, C_B, C_IPKT, C_IBYT]
FEEDBACK_NCOLS = 22


def convert_feedback_row(row: str) -> Optional[str]:
    """flow_scores.csv row -> 27-field flow row (flow_pre_lda.scala:146-248 convert_feedback_row_to_flow_row).

    Unused columns become "##"; hour/minute/second come from tstart "YYYY-MM-DD HH:MM:SS".
    Returns None for a malformed tstart (the reference would throw)."""
    f = row.split(",")
    try:
        hms = f[1].split(" ")[1].split(":")
        hour, mnt, sec = hms[0], hms[1], hms[2]
    except IndexError:
        return None
    out = ["##"] * NCOLS
    out[C_HOUR], out[C_MIN], out[C_SEC] = hour, mnt, sec
    out[C_IPKT], out[C_IBYT] = f[8], f[9]
    out[10], out[11] = f[4], f[5]
    out[C_SIP], out[C_DIP] = f[2], f[3]
    return ",".join(out)


def _java_split_len(line: str, sep: str = ",") -> int:
    parts = line.split(sep)
    while parts and parts[-1] == "":
        parts.pop()
    return len(parts) if line else 1


def read_flow_feedback(path: str) -> List[str]:
    """Rows of flow_scores.csv flagged non-threatening (sev == 3), converted to flow rows.

    Header dropped; rows must have 22 fields (Java split) and an integer severity
    field equal to 3 (flow_pre_lda.scala:258)."""
    if not os.path.exists(path):
        return []
    with open(path, "r", encoding="utf-8", newline="") as fh:
        lines = fh.read().split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    out = []
    for l in lines[1:]:
        l = l.rstrip("\r")
        if _java_split_len(l) != FEEDBACK_NCOLS:
            continue
        try:
            sev = int(l.split(",")[0])
        except ValueError:
            continue
        if sev == 3:
            r = convert_feedback_row(l)
            if r is not None:
                out.append(r)
    return out


@dataclass
class FlowTable:
    """Ingested flow rows (host) with per-row weights; feedback rows come last."""
    table: object               # _oninative.TextTable
    n_raw: int
    n_feedback: int
    dupfactor: int

    @property
    def n(self) -> int:
        return self.n_raw + self.n_feedback

    @property
    def ip_names(self) -> List[str]:
        """The IP dictionary's names (built once: config 5's is millions of strings, read by lda_pre,
        the post stage's row map and the scorer)."""
        names = self.__dict__.get("_ip_names")
        if names is None:
            names = self.__dict__["_ip_names"] = self.table.dict_names(0)
        return names

    def stats(self) -> dict:
        t = self.table
        return dict(rows=self.n, raw_rows=self.n_raw, feedback_rows=self.n_feedback, dropped_field_count=t.n_bad_fields,
                    dropped_non_numeric=t.n_bad_numeric, header_lines=t.n_header)


def list_inputs(path_spec: str) -> List[str]:
    """FLOW_PATH may be a file, a directory (all regular files, sorted) or a comma-separated list."""
    out = []
    for p in [x for x in path_spec.split(",") if x]:
        if os.path.isdir(p):
            out.extend(sorted(os.path.join(p, f) for f in os.listdir(p)
                              if not f.startswith((".", "_")) and os.path.isfile(os.path.join(p, f))))
        else:
            out.append(p)
    return out


def load_flow(flow_path: str, feedback_path: Optional[str] = None, dupfactor: int = 1000, threads: int = 8) -> FlowTable:
    t = native.lib().TextTable(NCOLS, NUMERIC, [[C_SIP, C_DIP]])
    paths = list_inputs(flow_path)
    if not paths:
        raise FileNotFoundError(f"no flow input under {flow_path!r}")
    t.load_files(paths, drop_header=True, threads=threads)
    n_raw = t.num_rows
    fb = read_flow_feedback(feedback_path) if feedback_path else []
    if fb:
        t.append_text("\n".join(fb), weight=int(dupfactor), threads=threads)
    return FlowTable(t, n_raw, t.num_rows - n_raw, int(dupfactor))
