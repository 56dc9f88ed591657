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

from .flow_io import (  # noqa: F401  (re-exported: the torch-free ingest)
    NCOLS, C_HOUR, C_MIN, C_SEC, C_SIP, C_DIP, C_A, C_B, C_IPKT, C_IBYT, NUMERIC, FEEDBACK_NCOLS,
    convert_feedback_row, _java_split_len, read_flow_feedback, FlowTable, list_inputs, load_flow)


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
        ok = p.index_select(0, i) == word_port if p.numel() else torch.zeros_like(word_port, dtype=torch.bool)
        return torch.where(ok, i, torch.full_like(i, -1))

    def decode(self, keys: np.ndarray) -> List[str]:
        """Word strings of ``keys``: one concatenation per word of a head ("[-1_]<port>_", one per
        (port, side)) and a tail ("<time>_<ibyt>_<ipkt>", one per bin triple), both built once
        (csrc/native/bind_native.cpp flow_word_names; ``decode_py`` is the Python form, its test oracle)."""
        from ..ops import native
        return native.lib().flow_word_names(np.asarray(self.ports, np.float64), self.NT, self.NB, self.NP,
                                            np.asarray(keys, np.int64))

    def decode_py(self, keys: np.ndarray) -> List[str]:
        k = np.asarray(keys, np.int64)
        prefix = k % 2
        k = k // 2
        nt = self.NT * self.NB * self.NP
        tail = k % nt                     # (tb * NB + bb) * NP + pb
        port = k // nt
        from ..ops import native
        pstr = native.lib().java_double_array(np.asarray(self.ports, np.float64))
        bstr = [java_double(float(i)) for i in range(max(self.NT, self.NB, self.NP))]
        heads = [h for ps in pstr for h in (f"{ps}_", f"-1_{ps}_")]
        tails = [f"{bstr[t]}_{bstr[b]}_{bstr[p]}" for t in range(self.NT) for b in range(self.NB)
                 for p in range(self.NP)]
        return [heads[h] + tails[t] for h, t in zip((port * 2 + prefix).tolist(), tail.tolist())]


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
    from ..ops import sortgroup as SG
    ports = SG.unique(feat.word_port).cpu().numpy()
    return FlowWordSpace(ports, len(feat.cuts["time"]) + 1, len(feat.cuts["ibyt"]) + 1, len(feat.cuts["ipkt"]) + 1)


def word_keys(feat: FlowFeatures, ws: FlowWordSpace):
    """(src_key, dst_key) int64 tensors; -1 where the port is not in the word space."""
    pid = ws.port_ids(feat.word_port)
    base_ok = pid >= 0
    src = ws.encode(pid.clamp_min(0), feat.time_bin, feat.ibyt_bin, feat.ipkt_bin, feat.src_prefix)
    dst = ws.encode(pid.clamp_min(0), feat.time_bin, feat.ibyt_bin, feat.ipkt_bin, feat.dst_prefix)
    neg = torch.full_like(src, -1)
    return torch.where(base_ok, src, neg), torch.where(base_ok, dst, neg)
