"""Netflow featurization: CSV -> per-event words -> (ip, word) counts.

Reference: flow_pre_lda.scala (pre-LDA) and flow_post_lda.scala:126-224 (the
same featurization repeated before scoring); SURVEY.md C4a-C4g, C5b.

Pipeline (MI355X):
  C++ TextTable ingest (27-col CSV, header rule, Java split/parseDouble)
  + analyst feedback rows (weight DUPFACTOR instead of 1000 copies)
  -> H2D of 7 numeric columns + 2 IP dictionary-id columns
  -> weighted ECDF cuts on device (time/ibyt deciles, ipkt quintiles)
  -> HIP `flow_words` kernel: time column, 3 bins, port case, "-1_" side
  -> int64 word keys  (port id, time bin, ibyt bin, ipkt bin, prefix)
  -> src/dest (ip, word) counts by sort-based group-by.
Word strings ("80.0_3.0_5.0_2.0", Java Double.toString of each part,
flow_pre_lda.scala:349) are only produced for the V distinct words.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..io.javafmt import java_double
from ..ops import native
from .quantiles import DECILES, QUINTILES, ecdf_cuts

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
        return self.table.dict_names(0)

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


class FlowWordSpace:
    """Integer word keys for flow words: key = ((((port*NT + tb)*NB + bb)*NP + pb)*2 + prefix).

    `ports` are the distinct word_port values (sorted float64); a key decodes to
    the reference word string "[-1_]<port>_<time_bin>_<ibyt_bin>_<ipkt_bin>" with
    every number in Java Double.toString form."""

    def __init__(self, ports: np.ndarray, n_time: int, n_ibyt: int, n_ipkt: int):
        self.ports = np.asarray(ports, np.float64)
        self.NT, self.NB, self.NP = int(n_time), int(n_ibyt), int(n_ipkt)
        if self.ports.size * self.NT * self.NB * self.NP * 2 >= (1 << 31):
            raise ValueError("flow word key space exceeds 31 bits")

    def encode(self, port_id, tb, bb, pb, prefix):
        return ((((port_id.to(torch.int64) * self.NT + tb.to(torch.int64)) * self.NB + bb.to(torch.int64)) * self.NP
                 + pb.to(torch.int64)) * 2 + prefix.to(torch.int64))

    def port_ids(self, word_port: torch.Tensor) -> torch.Tensor:
        """Index of each value in `ports` (-1 if absent)."""
        p = torch.from_numpy(self.ports).to(word_port.device)
        i = torch.searchsorted(p, word_port).clamp_max(max(p.numel() - 1, 0))
        ok = p[i] == word_port if p.numel() else torch.zeros_like(word_port, dtype=torch.bool)
        return torch.where(ok, i, torch.full_like(i, -1))

    def decode(self, keys: np.ndarray) -> List[str]:
        k = np.asarray(keys, np.int64)
        prefix = k % 2
        k = k // 2
        pb = k % self.NP
        k = k // self.NP
        bb = k % self.NB
        k = k // self.NB
        tb = k % self.NT
        port = k // self.NT
        from ..ops import native
        pstr = native.lib().java_double_array(np.asarray(self.ports, np.float64))
        bstr = [java_double(float(i)) for i in range(max(self.NT, self.NB, self.NP))]
        return [("-1_" if pr else "") + f"{pstr[po]}_{bstr[t]}_{bstr[b]}_{bstr[p]}"
                for pr, po, t, b, p in zip(prefix.tolist(), port.tolist(), tb.tolist(), bb.tolist(), pb.tolist())]


@dataclass
class FlowFeatures:
    """Per-row features on the device (rows = the FlowTable rows in `rows`, or all)."""
    time: torch.Tensor          # f64 col 27
    time_bin: torch.Tensor      # int8 col 30
    ibyt_bin: torch.Tensor      # int8 col 28
    ipkt_bin: torch.Tensor      # int8 col 29
    word_port: torch.Tensor     # f64 col 31
    src_prefix: torch.Tensor    # int8
    dst_prefix: torch.Tensor    # int8
    sip: torch.Tensor           # int32 ip dictionary ids
    dip: torch.Tensor
    weight: torch.Tensor        # int64
    cuts: Dict[str, np.ndarray] = field(default_factory=dict)
    rows: Optional[np.ndarray] = None   # table row index of each feature row


def _flow_words(cols, cuts, device):
    """HIP kernel on GPU; the vectorised torch transcription elsewhere (CPU pipeline / tests)."""
    from ..ops import hip as H
    if device.type == "cuda":
        return H.flow_words(cols["hour"], cols["minute"], cols["second"], cols["a"], cols["b"], cols["ipkt"],
                            cols["ibyt"], cuts["time"], cuts["ibyt"], cuts["ipkt"])
    from ..ops.reference import flow_words as ref
    return ref(cols["hour"], cols["minute"], cols["second"], cols["a"], cols["b"], cols["ipkt"], cols["ibyt"],
               cuts["time"], cuts["ibyt"], cuts["ipkt"])


def featurize(ft: FlowTable, device, cuts: Optional[Dict[str, np.ndarray]] = None, raw_only: bool = False) -> FlowFeatures:
    """Compute times, cuts (unless given), bins and word parts for the table rows.

    raw_only=True featurizes only the raw input rows (post-LDA stage: the
    reference re-reads FLOW_PATH without feedback, flow_post_lda.scala:126-137)."""
    device = torch.device(device)
    t = ft.table
    n = ft.n_raw if raw_only else ft.n
    def col(c):
        return torch.from_numpy(t.numeric(c)[:n]).to(device)
    cols = dict(hour=col(C_HOUR), minute=col(C_MIN), second=col(C_SEC), a=col(C_A), b=col(C_B), ipkt=col(C_IPKT),
                ibyt=col(C_IBYT))
    w = torch.from_numpy(t.weights()[:n].astype(np.int64)).to(device)
    if cuts is None:
        time = (cols["hour"] + cols["minute"] / 60) + cols["second"] / 3600
        cuts_t = dict(time=ecdf_cuts(time, DECILES, w), ibyt=ecdf_cuts(cols["ibyt"], DECILES, w),
                      ipkt=ecdf_cuts(cols["ipkt"], QUINTILES, w))
    else:
        cuts_t = {k: torch.as_tensor(np.asarray(v, np.float64), device=device) for k, v in cuts.items()}
    out = _flow_words(cols, cuts_t, device)
    return FlowFeatures(
        time=out["time"], time_bin=out["time_bin"], ibyt_bin=out["ibyt_bin"], ipkt_bin=out["ipkt_bin"],
        word_port=out["word_port"], src_prefix=out["src_prefix"], dst_prefix=out["dst_prefix"],
        sip=torch.from_numpy(t.dict_ids(C_SIP)[:n]).to(device), dip=torch.from_numpy(t.dict_ids(C_DIP)[:n]).to(device),
        weight=w, cuts={k: v.cpu().numpy() for k, v in cuts_t.items()}, rows=np.arange(n, dtype=np.int64))


def word_space_for(feat: FlowFeatures) -> FlowWordSpace:
    ports = torch.unique(feat.word_port).cpu().numpy()
    return FlowWordSpace(ports, len(feat.cuts["time"]) + 1, len(feat.cuts["ibyt"]) + 1, len(feat.cuts["ipkt"]) + 1)


def word_keys(feat: FlowFeatures, ws: FlowWordSpace):
    """(src_key, dst_key) int64 tensors; -1 where the port is not in the word space."""
    pid = ws.port_ids(feat.word_port)
    base_ok = pid >= 0
    src = ws.encode(pid.clamp_min(0), feat.time_bin, feat.ibyt_bin, feat.ipkt_bin, feat.src_prefix)
    dst = ws.encode(pid.clamp_min(0), feat.time_bin, feat.ibyt_bin, feat.ipkt_bin, feat.dst_prefix)
    neg = torch.full_like(src, -1)
    return torch.where(base_ok, src, neg), torch.where(base_ok, dst, neg)
