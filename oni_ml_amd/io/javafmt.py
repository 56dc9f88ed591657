"""Pure-Python versions of the reference's number-to-text conversions.

* ``java_double`` - java.lang.Double.toString (shortest round-trip digits,
  decimal for 1e-3 <= |x| < 1e7, otherwise ``d.dddE<exp>``).  Used for flow
  words (flow_pre_lda.scala:349), the time column and the scores.
* ``py2_float``   - Python 2 ``str(float)`` ("%.12g", ".0" appended when the
  text looks integral), used by lda_post.py for doc_results / word_results.

The C++ runtime (csrc/native/fmt.h) implements the same functions for bulk
output; these are the oracles the tests compare it against.
"""
from __future__ import annotations

import math


def java_double(x: float) -> str:
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    r = repr(abs(x))  # shortest round-trip
    mant, _, exp = r.partition("e")
    e = int(exp) if exp else 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # decimal exponent of the first significant digit
    if ip.strip("0"):
        e10 = len(ip.lstrip("0")) - 1 + e
    else:
        lead = len(fp) - len(fp.lstrip("0"))
        e10 = -lead - 1 + e
    digits = digits.rstrip("0") or "0"
    sign = "-" if x < 0 else ""
    a = abs(x)
    if 1e-3 <= a < 1e7:
        if e10 >= 0:
            ipart = digits[: e10 + 1].ljust(e10 + 1, "0")
            fpart = digits[e10 + 1:] or "0"
        else:
            ipart = "0"
            fpart = "0" * (-e10 - 1) + digits
        return f"{sign}{ipart}.{fpart}"
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{e10}"


def py2_float(x: float) -> str:
    x = float(x)
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    s = "%.12g" % x
    if "." not in s and "e" not in s:
        s += ".0"
    return s


def java_int_double(i: int) -> str:
    """Scala `i.toDouble.toString` for a small integer (bins in flow words): '3.0'."""
    return java_double(float(i))
