"""lda_pre / lda_post equivalents against literal transcriptions of the reference scripts."""
import numpy as np
import pytest
import torch

from oni_ml_amd.corpus.builder import DocWordCounts, concat, count_pairs, lda_pre, lda_pre_reference, read_doc_wc
from oni_ml_amd.corpus.csr import Corpus
from oni_ml_amd.export import lda_post
from oni_ml_amd.io import ldac

from . import oracles as O


def _random_dwc(rng, n=400, ndocs=40, nwords=60):
    doc = torch.from_numpy(rng.integers(0, ndocs, n))
    word = torch.from_numpy(rng.integers(0, nwords, n))
    cnt = torch.from_numpy(rng.integers(1, 9, n))
    return DocWordCounts(doc, word, cnt)


def test_lda_pre_matches_script():
    rng = np.random.default_rng(0)
    dwc = _random_dwc(rng)
    built = lda_pre(dwc)
    lines = [(f"ip{d}", f"w{w}", c) for d, w, c in zip(dwc.doc.tolist(), dwc.word.tolist(), dwc.count.tolist())]
    words, docs, model = lda_pre_reference(lines)
    assert [f"w{k}" for k in built.word_keys.tolist()] == words
    assert [f"ip{k}" for k in built.doc_keys.tolist()] == docs
    c = built.corpus
    got = []
    for d in range(c.num_docs):
        a, b = c.doc_ptr[d], c.doc_ptr[d + 1]
        got.append("%d%s" % (b - a, "".join(" %d:%d" % (w, n) for w, n in zip(c.word_idx[a:b], c.counts[a:b]))))
    assert got == model


def test_count_pairs_and_sections():
    doc = torch.tensor([1, 1, 2, 1, 2])
    word = torch.tensor([5, 5, 7, 6, 7])
    w = torch.tensor([1, 1, 1, 1000, 1])
    p = count_pairs(doc, word, w)
    assert list(zip(p.doc.tolist(), p.word.tolist(), p.count.tolist())) == [(1, 5, 2), (1, 6, 1000), (2, 7, 2)]
    both = concat([p, p])
    assert both.n == 6
    merged = concat([p, p], merge=True)
    assert merged.count.tolist() == [4, 2000, 4]


def test_doc_wc_file_roundtrip(tmp_path):
    p = tmp_path / "doc_wc.dat"
    p.write_text("10.0.0.1,80.0_1.0_2.0_3.0,4\n10.0.0.2,53.0_0.0_0.0_0.0,1\n10.0.0.1,53.0_0.0_0.0_0.0,2\n")
    dwc, ips, words = read_doc_wc(str(p))
    built = lda_pre(dwc)
    assert [ips[i] for i in built.doc_keys] == ["10.0.0.1", "10.0.0.2"]
    assert [words[i] for i in built.word_keys] == ["80.0_1.0_2.0_3.0", "53.0_0.0_0.0_0.0"]
    c = built.corpus
    assert c.doc_ptr.tolist() == [0, 2, 3] and c.word_idx.tolist() == [0, 1, 1] and c.counts.tolist() == [4, 2, 1]


def test_model_dat_roundtrip(tmp_path):
    c = Corpus.from_docs([[(0, 3), (2, 1)], [(1, 5)], [(2, 2), (0, 1), (3, 7)]])
    ldac.write_model_dat(str(tmp_path / "model.dat"), c)
    assert (tmp_path / "model.dat").read_text().splitlines() == ["2 0:3 2:1", "1 1:5", "3 2:2 0:1 3:7"]
    c2 = ldac.read_model_dat(str(tmp_path / "model.dat"))
    assert np.array_equal(c2.doc_ptr, c.doc_ptr) and np.array_equal(c2.word_idx, c.word_idx) and c2.num_terms == 4


def test_doc_results_matches_lda_post(tmp_path):
    rng = np.random.default_rng(1)
    g = rng.random((30, 20)) * 10
    g[3] = 0.0
    names = [f"10.1.0.{i}" for i in range(30)]
    ldac.save_gamma(str(tmp_path / "final.gamma"), g)
    gtext = (tmp_path / "final.gamma").read_text().splitlines()
    th = lda_post.doc_topics(g, strict=True)
    lda_post.write_doc_results(str(tmp_path / "doc_results.csv"), names, th)
    got = (tmp_path / "doc_results.csv").read_text().splitlines()
    want = [O.lda_post_doc_line(n, line) for n, line in zip(names, gtext)]
    assert got == want


def test_word_results_matches_lda_post(tmp_path):
    rng = np.random.default_rng(2)
    K, V = 20, 50
    lb = np.log(rng.random((K, V)))
    lb[:, 7] = -100.0
    ldac.save_beta(str(tmp_path / "final.beta"), lb)
    words = np.loadtxt(str(tmp_path / "final.beta"), np.float64)      # lda_post.py:70
    names = [f"{p}.0_{i % 11}.0_{i % 7}.0_{i % 5}.0" for i, p in enumerate([80, 333333, 111111, 443, 53] * 10)]
    names[3] = "-1_" + names[3]
    phi = lda_post.word_topics(lb, strict=True)
    lda_post.write_word_results(str(tmp_path / "word_results.csv"), lda_post.truncate_s20(names), phi)
    got = (tmp_path / "word_results.csv").read_text().splitlines()
    # literal lda_post.py:88-122
    p_wgz = np.empty([words.shape[1], words.shape[0]])
    for col, w in enumerate(words):
        raw = [np.exp(wi) for wi in w]
        tot = 0
        for r in raw:
            tot = tot + r
        p_wgz[:, col] = [r / tot for r in raw]
    want = []
    for j in range(V):
        nm = names[j].encode()[:20].decode()
        want.append(nm + "," + " ".join(O.py2(x) for x in p_wgz[j]))
    assert got == want
    keys, vals = lda_post.read_results(str(tmp_path / "word_results.csv"))
    assert keys[0] == names[0][:20] and vals.shape == (V, K)


def test_strict_requires_20_topics():
    with pytest.raises(ValueError):
        lda_post.check_strict_k(10, True)
    lda_post.check_strict_k(10, False)


def test_export_read_back_equals_text_roundtrip(tmp_path):
    """lda_post export with read_back: the values handed to the scorers equal the files parsed back
    (Python-2 str text -> strtod), bit for bit, and the files are unchanged by the option."""
    from oni_ml_amd.export import lda_post
    from oni_ml_amd.ops import native
    rng = np.random.default_rng(3)
    g = rng.random((300, 20)) * 50
    lb = np.log(rng.random((20, 700)) / 700)
    dn = [f"10.0.{i // 256}.{i % 256}" for i in range(300)]
    wn = [f"{i}_80_1_2_3" for i in range(700)]
    th, ph, _ = lda_post.export(dn, g, wn, lb, str(tmp_path / "d.csv"), str(tmp_path / "w.csv"), read_back=True)
    d1, w1 = (tmp_path / "d.csv").read_text(), (tmp_path / "w.csv").read_text()
    th0, ph0, _ = lda_post.export(dn, g, wn, lb, str(tmp_path / "d.csv"), str(tmp_path / "w.csv"))
    assert (tmp_path / "d.csv").read_text() == d1 and (tmp_path / "w.csv").read_text() == w1
    N = native.lib()
    assert np.array_equal(th, N.roundtrip_py2(np.ascontiguousarray(th0)))
    assert np.array_equal(ph, N.roundtrip_py2(np.ascontiguousarray(ph0)))
    _, tv = lda_post.read_results(str(tmp_path / "d.csv"))
    assert np.array_equal(tv, th)


def test_export_deferred_matches_read_back_export(tmp_path):
    """export_deferred: the same files, and the round-trip tables bitwise equal to the writer's read-back."""
    import numpy as np
    from oni_ml_amd.export import lda_post
    rng = np.random.default_rng(5)
    D, V, K = 300, 200, 20
    gamma = rng.gamma(0.3, 2.0, (D, K)) + 1e-3
    gamma[3] = 0.0
    lb = np.log(rng.dirichlet(np.full(V, 0.1), K))
    docs = [f"10.0.{i // 256}.{i % 256}" for i in range(D)]
    words = [f"{i}_80_tcp_{'x' * (i % 30)}" for i in range(V)]
    for strict in (True, False):
        a = tmp_path / f"a{strict}"
        b = tmp_path / f"b{strict}"
        a.mkdir(), b.mkdir()
        th, ph, wn = lda_post.export(docs, gamma, words, lb, str(a / "d.csv"), str(a / "w.csv"), strict=strict,
                                     read_back=True)
        th2, ph2, wn2, join = lda_post.export_deferred(docs, gamma, words, lb, str(b / "d.csv"), str(b / "w.csv"),
                                                       strict=strict)
        join()
        assert np.array_equal(th, th2) and np.array_equal(ph, ph2) and wn == wn2
        for f in ("d.csv", "w.csv"):
            assert (a / f).read_bytes() == (b / f).read_bytes()
