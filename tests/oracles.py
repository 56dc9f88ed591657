"""Tiny literal Python transcriptions of the reference's Scala semantics (test oracles only).

Each function mirrors one Scala definition line by line so the vectorised /
native implementations can be checked against it on small random inputs.
"""
import math

from oni_ml_amd.io.javafmt import java_double


def java_split(s, sep=","):
    parts = s.split(sep)
    if s == "":
        return [""]
    while parts and parts[-1] == "":
        parts.pop()
    return parts


def add_time(row):
    """flow_pre_lda.scala:272-277"""
    return float(row[4]) + float(row[5]) / 60 + float(row[6]) / 3600


def bin_count(v, cuts):
    b = 0
    for c in cuts:
        if v > c:
            b += 1
    return b


def adjust_port(a, b, time_bin, ibyt_bin, ipkt_bin):
    """flow_pre_lda.scala:317-362 with dport = col 10 (a), sport = col 11 (b). Returns (word_port, src, dest)."""
    dport, sport = float(a), float(b)
    word_port = 111111.0
    if (dport <= 1024 or sport <= 1024) and (dport > 1024 or sport > 1024) and min(dport, sport) != 0:
        p_case = 2
        word_port = min(dport, sport)
    elif dport > 1024 and sport > 1024:
        p_case = 3
        word_port = 333333.0
    elif dport == 0 and sport != 0:
        word_port = sport
        p_case = 4
    elif sport == 0 and dport != 0:
        word_port = dport
        p_case = 4
    else:
        p_case = 1
        word_port = max(dport, sport) if min(dport, sport) == 0 else 111111.0
    word = "_".join(java_double(x) for x in (word_port, float(time_bin), float(ibyt_bin), float(ipkt_bin)))
    src = dest = word
    if p_case == 2 and dport < sport:
        dest = "-1_" + dest
    elif p_case == 2 and sport < dport:
        src = "-1_" + src
    elif p_case == 4 and dport == 0:
        src = "-1_" + src
    elif p_case == 4 and sport == 0:
        dest = "-1_" + dest
    return word_port, src, dest


def extract_subdomain(url, country_codes):
    """dns_pre_lda.scala:185-220 -> [domain, subdomain, subdomain.length, num.periods]"""
    spliturl = java_split(url, ".")
    if url and all(p == "" for p in url.split(".")):
        spliturl = []
    numparts = len(spliturl)
    domain = "None"
    subdomain = "None"
    is_ip = ("IP" if (spliturl[numparts - 1] == "arpa" and spliturl[numparts - 2] == "in-addr") else "Name") \
        if numparts > 2 else "Unknown"
    if numparts > 2 and is_ip != "IP":
        if spliturl[numparts - 1] in country_codes:
            domain = spliturl[numparts - 3]
            if 1 <= numparts - 3:
                subdomain = ".".join(spliturl[0:numparts - 3])
        else:
            domain = spliturl[numparts - 2]
            if 1 <= numparts - 2:
                subdomain = ".".join(spliturl[0:numparts - 2])
    return [domain, subdomain, str(len(subdomain)) if subdomain != "None" else "0", str(numparts)]


def entropy_any_order(v):
    """dns_pre_lda.scala:278-284 up to summation order."""
    counts = {}
    for ch in v:
        counts[ch] = counts.get(ch, 0) + 1
    s = 0.0
    for c in counts.values():
        p = c / len(v)
        s += -p * math.log10(p) / math.log10(2)
    return s


def lda_post_doc_line(ip, gamma_row_text):
    """lda_post.py:35-59 for one final.gamma line (Python 3 rendition of the Python 2 code)."""
    t = [float(x) for x in gamma_row_text.split(" ")]
    total = 0
    for x in t:
        total = total + x
    if total > 0:
        norm = " ".join(py2(x / total) for x in t)
    else:
        norm = " ".join(["0.0"] * 20)
    return "%s,%s" % (ip, norm)


def py2(x):
    s = "%.12g" % x
    if "." not in s and "e" not in s and "n" not in s:
        s += ".0"
    return s
