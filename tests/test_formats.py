"""Text formats: Java Double.toString, Python-2 str(float), lda-c %5.10f, Java parseDouble, CSV ingest rules."""
import math
import os
import random
import struct

import numpy as np
import pytest

from oni_ml_amd.io.javafmt import java_double, py2_float
from oni_ml_amd.ops import native

N = native.lib()


@pytest.mark.parametrize("x,s", [
    (80.0, "80.0"), (0.05, "0.05"), (1e-20, "1.0E-20"), (1234567.0, "1234567.0"), (1e7, "1.0E7"),
    (12345678.0, "1.2345678E7"), (0.001, "0.001"), (0.0001, "1.0E-4"), (-0.0, "-0.0"), (0.0, "0.0"),
    (23.983333333333334, "23.983333333333334"), (333333.0, "333333.0"), (float("nan"), "NaN"),
    (float("inf"), "Infinity"), (-1.5e-300, "-1.5E-300"), (9999999.0, "9999999.0"),
])
def test_java_double_known(x, s):
    assert java_double(x) == s
    assert N.java_double(x) == s


def test_java_double_native_matches_python_random():
    rng = random.Random(1)
    vals = []
    for _ in range(20000):
        v = struct.unpack("d", struct.pack("Q", rng.getrandbits(64)))[0]
        if v == v:
            vals.append(v)
        vals.append(rng.random() * 10 ** rng.randint(-12, 12))
    for v in vals:
        assert N.java_double(v) == java_double(v), v
        assert float(java_double(v).replace("E", "e")) == v


@pytest.mark.parametrize("x,s", [(1 / 3, "0.333333333333"), (1.0, "1.0"), (1e-5, "1e-05"), (0.05, "0.05"),
                                 (123456789012345.0, "1.23456789012e+14"), (0.0, "0.0"), (5e-324, "4.94065645841e-324")])
def test_py2_float(x, s):
    assert py2_float(x) == s
    assert N.py2_float(x) == s


def test_roundtrips():
    a = np.array([1 / 3, -100.0, 2.5e-11, 0.123456789012345678])
    assert np.array_equal(N.roundtrip_fixed10(a), np.array([float("%5.10f" % x) for x in a]))
    assert np.array_equal(N.roundtrip_py2(a), np.array([float(py2_float(x)) for x in a]))


@pytest.mark.parametrize("s,v", [(" 12.5 ", 12.5), ("1e3", 1000.0), ("5d", 5.0), ("-2", -2.0), ("+7", 7.0),
                                 (".5", 0.5), ("NaN", None), ("##", None), ("", None), ("abc", None)])
def test_java_parse(s, v):
    r = N.java_parse_double(s)
    if s == "NaN":
        assert r != r
    elif v is None:
        assert r is None
    else:
        assert r == v


def test_table_ingest_rules(tmp_path):
    hdr = "a,b,c,d"
    lines = [
        hdr,
        "1,2,x,4",           # ok
        "  5,6,y,7  ",        # trimmed
        "1,2,3",             # 3 fields -> dropped
        "1,2,3,4,",          # trailing empty field vanishes -> 4 fields, kept as "1,2,3,4"
        "1,2,,4",            # empty middle field kept (non-numeric col 2 is a string col)
        "q,2,x,4",           # non-numeric col 0 -> dropped
        hdr,                 # every header copy dropped
        "8,9,z,10\r",        # CRLF
        "",
    ]
    p = tmp_path / "in.csv"
    p.write_text("\n".join(lines) + "\n")
    t = N.TextTable(4, [0, 1, 3], [[2]])
    t.load_files([str(p)], drop_header=True, threads=2)
    assert t.num_rows == 5
    assert [t.row_text(i) for i in range(t.num_rows)] == ["1,2,x,4", "5,6,y,7", "1,2,3,4", "1,2,,4", "8,9,z,10"]
    assert t.numeric(0).tolist() == [1, 5, 1, 1, 8]
    assert t.dict_names(0) == ["x", "y", "3", "", "z"]
    assert t.n_header == 2 and t.n_bad_numeric == 1 and t.n_bad_fields == 2
    t.append_text("3,3,x,3", weight=1000)
    assert t.weights().tolist() == [1, 1, 1, 1, 1, 1000]
    assert t.dict_ids(2).tolist()[-1] == 0


def test_table_ingest_thread_invariance(tmp_path):
    rng = np.random.default_rng(0)
    n = 60000
    names = [f"10.0.{i // 256}.{i % 256}" for i in range(3000)]
    rows = [f"{rng.integers(0, 100)},{names[rng.integers(0, 3000)]},{names[rng.integers(0, 3000)]}" for _ in range(n)]
    p = tmp_path / "big.csv"
    p.write_text("h,s,d\n" + "\n".join(rows) + "\n")
    outs = []
    for th in (1, 7):
        t = N.TextTable(3, [0], [[1, 2]])
        t.load_files([str(p)], drop_header=True, threads=th)
        outs.append((t.numeric(0).tolist(), t.dict_ids(1).tolist(), t.dict_ids(2).tolist(), t.dict_names(0)))
    assert outs[0] == outs[1]


def test_table_numbers_and_long_names(tmp_path):
    """Numeric fields through the exact short-number path (<= 15 digits, one '.') and the general
    parse agree with a correctly rounded parse; names longer than the inline 16 key bytes (sharing a
    16-byte prefix) stay distinct; lines of every length around the 32-byte scan blocks."""
    rng = np.random.default_rng(5)
    vals, lines = [], ["h,n,s"]
    for i in range(4000):
        nd = int(rng.integers(1, 19))
        digits = "".join(str(d) for d in rng.integers(0, 10, nd))
        dot = int(rng.integers(0, nd + 1))
        txt = digits[:dot] + "." + digits[dot:] if rng.random() < 0.7 else digits
        txt = ("-" if rng.random() < 0.2 else "") + txt
        if txt in (".", "-."):
            txt = "0"
        vals.append(float(txt))
        pad = "x" * int(rng.integers(1, 40))
        name = "prefix-sixteen-b" + str(i % 97) if i % 3 == 0 else f"10.{i % 5}.{i % 7}.{pad[:3]}"
        lines.append(f"{txt},{name},{pad}")
    for txt in ["5.", ".5", "-0", "1e5", "2.5E-3", "7d", "+3", "0.1000000000000000055511151231257827"]:
        vals.append(float(txt.rstrip("d")))
        lines.append(f"{txt},z,q")
    p = tmp_path / "nums.csv"
    p.write_text("\n".join(lines) + "\n")
    for th in (1, 5):
        t = N.TextTable(3, [0], [[1]])
        t.load_files([str(p)], drop_header=True, threads=th)
        got = t.numeric(0)
        assert t.num_rows == len(vals)
        assert got.tolist() == vals
        assert np.array_equal(np.signbit(got), np.signbit(np.array(vals)))
        names = t.dict_names(0)
        ids = t.dict_ids(1)
        assert [names[j] for j in ids.tolist()] == [ln.split(",")[1] for ln in lines[1:]]


def test_writer_kinds(tmp_path):
    t = N.TextTable(2, [0], [[1]])
    p = tmp_path / "t.csv"
    p.write_text("1,a\n2,b\n3,c\n")
    t.load_files([str(p)], drop_header=False)
    out = tmp_path / "o.csv"
    order = np.array([2, 0], np.int64)
    N.write_rows(str(out), None, [("table", t, order), ("java", np.array([1e-20, 80.0])),
                                  ("int", np.array([3, 4])), ("dict", ["x", "y"], np.array([1, 0], np.int32)),
                                  ("pair", ["10.0.0.2", "10.0.0.10"], np.array([0, 1], np.int32), np.array([1, 0], np.int32)),
                                  ("py2row", np.array([[1 / 3, 0.5], [1.0, 2.0]]), " "), ("const", "k")], n=2)
    assert out.read_text().splitlines() == [
        "3,c,1.0E-20,3,y,10.0.0.10 10.0.0.2,0.333333333333 0.5,k",
        "1,a,80.0,4,x,10.0.0.10 10.0.0.2,1.0 2.0,k",
    ]


def test_ldac_files_roundtrip(tmp_path):
    from oni_ml_amd.io import ldac
    lb = np.array([[-1.5, -100.0, -0.25], [-2.0, -3.0, -4.0]])
    ldac.save_model(str(tmp_path / "final"), lb, 0.1234)
    txt = (tmp_path / "final.beta").read_text().splitlines()
    assert txt[0] == " -1.5000000000 -100.0000000000 -0.2500000000"
    lb2, a = ldac.load_model(str(tmp_path / "final"))
    assert np.array_equal(lb, lb2) and a == pytest.approx(0.1234)
    g = np.array([[1.0, 2.5], [3.25, 0.125]])
    ldac.save_gamma(str(tmp_path / "final.gamma"), g)
    assert (tmp_path / "final.gamma").read_text() == "1.0000000000 2.5000000000\n3.2500000000 0.1250000000\n"
    assert ldac.format_likelihood_line(-12345.678, 0.00123) == "-12345.6780000000\t1.23000e-03\n"
    assert ldac.format_likelihood_line(-1.0, math.inf) == "-1.0000000000\t  inf\n"


def _edge_values(n=20000, seed=3):
    rng = np.random.default_rng(seed)
    v = np.concatenate([
        rng.uniform(-120, 30, n), -100.0 * np.ones(4), np.ldexp(rng.integers(0, 1 << 20, n).astype(np.float64),
                                                                -rng.integers(0, 45, n)),
        [0.0, -0.0, -1e-12, 1e-12, 0.5e-10, -0.5e-10, 2.0 ** -11, -(2.0 ** -11), 1e15, -3.3e19, 123456789.0000000005,
         5e-324, 1.7976931348623157e308],
        rng.standard_normal(n) * 1e-6,
    ])
    return v


def test_fixed10_and_py2_match_printf(tmp_path):
    """The C++ writers' "%5.10f" (lda-c .beta/.gamma) and "%.12g" (Python-2 str) equal C printf exactly,
    including ties, tiny negatives (-0.0000000000), huge and subnormal values."""
    v = _edge_values()
    p = tmp_path / "g.txt"
    native.lib().write_rows(str(p), None, [("fixedrow", v.reshape(1, -1), " ")], n=1)
    got = p.read_text().rstrip("\n").split(" ")
    assert got == ["%5.10f" % x for x in v]
    p2 = tmp_path / "p.txt"
    native.lib().write_rows(str(p2), None, [("py2row", v.reshape(-1, 1), " ")], n=v.size)
    want = []
    for x in v:
        s = "%.12g" % x
        want.append(s if ("." in s or "e" in s or "n" in s) else s + ".0")
    assert p2.read_text().splitlines() == want


def test_wide_rows_thread_invariant(tmp_path):
    """A K x V .beta file (few, very wide rows) is split over threads; output is identical to 1 thread."""
    lb = np.random.default_rng(0).uniform(-100, 0, (7, 70_001))   # >= 2^16 wide: the per-row segment path
    a, b = tmp_path / "a.beta", tmp_path / "b.beta"
    native.lib().write_rows(str(a), None, [("const", ""), ("fixedrow", lb, " ")], sep=" ", n=7, threads=1)
    native.lib().write_rows(str(b), None, [("const", ""), ("fixedrow", lb, " ")], sep=" ", n=7, threads=8)
    assert a.read_bytes() == b.read_bytes()
    assert np.allclose(np.loadtxt(str(a)), lb, atol=1e-10)


def test_ldac_corpus_text_native(tmp_path):
    """model.dat writer/reader (C++, multithreaded): python-formatted equality, blank lines, bad lines."""
    from oni_ml_amd.corpus.csr import Corpus
    from oni_ml_amd.io import ldac
    rng = np.random.default_rng(1)
    lens = rng.zipf(1.6, 30_000).clip(1, 3000)
    ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    w = rng.integers(0, 9000, ptr[-1]).astype(np.int32)
    c = rng.integers(1, 5000, ptr[-1]).astype(np.int64)
    p = tmp_path / "model.dat"
    ldac.write_model_dat(str(p), Corpus(ptr, w, c, 9000))
    lines = p.read_text().splitlines()
    assert len(lines) == lens.size
    for d in (0, 1, 777, lens.size - 1):
        a, b = ptr[d], ptr[d + 1]
        assert lines[d] == " ".join([str(b - a)] + [f"{x}:{y}" for x, y in zip(w[a:b], c[a:b])])
    r = ldac.read_model_dat(str(p))
    assert np.array_equal(r.doc_ptr, ptr) and np.array_equal(r.word_idx, w) and np.array_equal(r.counts, c)
    assert r.num_terms == int(w.max()) + 1
    q = tmp_path / "m2.dat"
    q.write_text("2 0:1 3:2\n\n1 5:7\r\n")
    r = ldac.read_model_dat(str(q))
    assert r.doc_ptr.tolist() == [0, 2, 3] and r.word_idx.tolist() == [0, 3, 5] and r.counts.tolist() == [1, 2, 7]
    q.write_text("3 0:1 3:2\n")
    with pytest.raises(RuntimeError, match="declares 3 entries"):
        ldac.read_model_dat(str(q))


@pytest.mark.parametrize("mode", [0, 1])
def test_fast_formatting_matches_exact(mode):
    """fmt.h's error-free-product fast paths ("%5.10f" and py2 "%.12g") against the exact
    printf-equivalent conversions: text and read-back value, over magnitudes, ties at both grids,
    carries, powers of ten, subnormals and raw bits."""
    N = native.lib()
    rng = np.random.default_rng(11 + mode)
    n = 300_000
    sets = [
        np.exp(rng.uniform(-700, 700, n)) * rng.choice([-1, 1], n),
        rng.random(n),
        np.log(rng.random(n)) * rng.uniform(0, 50, n),
        rng.integers(-10**13, 10**13, n) / 10.0 ** rng.integers(0, 16, n),
        (rng.integers(0, 10**9, n) * 2 + 1) / 2e10,                                # %.10f midpoints
        (rng.integers(10**11, 10**12, n) * 10 + 5) / 10.0 ** rng.integers(5, 20, n),  # %.12g midpoints
        rng.integers(0, 2**63, n, dtype=np.uint64).view(np.float64),
        rng.random(n) * 1e-8,
        np.ldexp(1.0, rng.integers(-60, 60, n)) * rng.integers(1, 2**20, n),            # dyadic: exact ties
        10.0 ** rng.integers(-12, 12, n) * (1 + rng.integers(-3, 4, n) * 2.0**-52),    # around powers of 10
        (10.0 ** rng.integers(1, 13, n) - 1) / 10.0 ** rng.integers(0, 14, n),          # 9...9 carries
        np.array([0.0, -0.0, 1.0, -1.0, 1e-9, -1e-9, 99999.99999999995, 1e5, 9.99999999999995e-10, 5e-324,
                  2.2250738585072014e-308, 2.225073858507201e-308, 1e300, 123456789012.5, 999999999999.5,
                  1e12, 1e-5, 1e-4, 0.5e-10, 1.5e-10]),
    ]
    for a in sets:
        a = a[np.isfinite(a)]
        assert N.fmt_selfcheck(a, mode) == (0, 0, -1)


def test_word_assignments_native_matches_loop(tmp_path):
    """word-assignments.dat (lda-c write_word_assignment: "%03d" then " %04d:%02d") from the device
    argmax + native writer equals the literal per-document loop, incl. words >= 10^4 and docs >= 10^3."""
    from oni_ml_amd.corpus.csr import Corpus
    from oni_ml_amd.models.lda.estimate import write_assignments, write_assignments_reference
    rng = np.random.default_rng(3)
    V, K = 12_000, 7
    lens = np.r_[rng.integers(1, 30, 200), [1500]]
    ptr = np.concatenate([[0], np.cumsum(lens)])
    words = np.concatenate([np.sort(rng.choice(V, n, replace=False)) for n in lens]).astype(np.int32)
    c = Corpus(ptr, words, np.ones(len(words), np.int64), V)
    log_beta = np.log(rng.dirichlet(np.ones(V), K))
    gamma = rng.gamma(2.0, 3.0, (len(lens), K))
    write_assignments(str(tmp_path / "a.dat"), c, log_beta, gamma)
    write_assignments_reference(str(tmp_path / "b.dat"), c, log_beta, gamma)
    a, b = (tmp_path / "a.dat").read_text(), (tmp_path / "b.dat").read_text()
    assert a == b
    assert a.splitlines()[-1].startswith("1500 ") and " 11" in a
