"""GPU parity of the packed tokenizer windows (short-document corpora).

The wave tokenizer indexes several consecutive short documents per window
(`k_tokenize_wave<true>`); no token, joiner (WB6/7, WB11/12) or '_' run may span
a document boundary, per-document TF/length/norm must equal the one-document
path, and packs that cannot take the packed path (window or term capacity,
empty or non-ASCII documents, replaced keys) go to the one-per-window pass.
Checked against the CPU oracle (`oracle/`) with the pack size forced through
`TFIDF_PACK_DOCS` and with the automatic choice.
"""
import random

import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

from test_gpu_parity import ALPHABET, assert_hits_equal

pytestmark = pytest.mark.gpu


def build_pair(texts, keys=None, cap_log2=18):
    g = ShardIndex(vocab_capacity_log2=cap_log2)
    g.add_documents(texts, keys)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(keys[i] if keys else str(i).encode(), t)
    o.commit()
    return g, o


def check_docs(g, o, n):
    s = g.stats()
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in range(n):
        assert g.doc_terms(d) == o.doc_terms(d), d
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d)), d


# documents whose edges would join across a boundary if the window ignored it
BOUNDARY_DOCS = [b"abc.", b"def", b"x_", b"_y", b"1,", b"2", b"don'", b"t", b"a:", b"b", b"3;", b"4",
                 b"end", b"start", b"tail ", b" head", b"___", b"w" * 12, b"w" * 12, b"Q", b"q",
                 b"k.", b".k", b"9", b"9", b"abcdefghij", b"abcdefghij", b"z" * 20, b"z" * 20]


@pytest.mark.parametrize("pack", [2, 5, 16])
def test_boundary_joiners_forced_pack(monkeypatch, pack):
    monkeypatch.setenv("TFIDF_PACK_DOCS", str(pack))
    texts = BOUNDARY_DOCS * 3
    g, o = build_pair(texts)
    assert g.stats()["pack_docs"] == pack
    check_docs(g, o, len(texts))
    for q in [b"abc", b"def", b"x_", b"dont", b"don't", b"t", b"12", b"1,2", b"q", b"k", b"99", b"z" * 20]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()


@pytest.mark.parametrize("pack", [3, 16])
def test_random_punctuation_short_docs(monkeypatch, pack):
    monkeypatch.setenv("TFIDF_PACK_DOCS", str(pack))
    rng = random.Random(pack)
    texts = ["".join(rng.choice(ALPHABET) for _ in range(rng.randint(1, 240))).encode() for _ in range(1500)]
    g, o = build_pair(texts)
    check_docs(g, o, len(texts))
    for q in [b"a", b"b.c x", b"3,14", b"abc xyz", b"y" * 3]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()


def test_auto_pack_short_zipf_docs_and_queries():
    texts = synth.corpus(6000, V=30000, len_min=20, len_max=90)
    g, o = build_pair(texts)
    s = g.stats()
    assert s["pack_docs"] > 1 and s["long_docs"] == 0
    check_docs(g, o, len(texts))
    qs = synth.queries(30, lo=1, hi=5000)
    for q in qs[:10]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    docs, scores, counts = g.search_batch(qs, 10)
    for i, q in enumerate(qs):
        got = list(zip(docs[i, :counts[i]].tolist(), scores[i, :counts[i]].tolist()))
        assert_hits_equal(got, o.search(q, 10))
    g.close()
    o.close()


def test_pack_retry_paths(monkeypatch):
    """Empty documents, a non-contiguous live map (replaced keys), a document
    too long for the window and over-full packs all reach the one-per-window
    pass and still equal the oracle."""
    monkeypatch.setenv("TFIDF_PACK_DOCS", "16")
    rng = random.Random(5)
    texts = synth.corpus(400, V=5000, len_min=5, len_max=60)
    texts[3] = b""
    texts[40] = b" ... "
    texts[77] = b" ".join(synth.word(r) for r in range(1, 1200))      # > 4 KB: long path
    texts[100:116] = [b" ".join(synth.word(rng.randint(1, 4000)) for _ in range(120)) for _ in range(16)]
    keys = [b"k%d" % i for i in range(350)] + [b"k%d" % (7 * j) for j in range(50)]   # every 7th replaced
    g, o = build_pair(texts, keys)
    s = g.stats()
    assert s["pack_docs"] == 16 and s["pack_retried"] > 0 and s["num_docs"] == o.num_docs == 350
    check_docs(g, o, 350)
    for q in synth.queries(10, lo=1, hi=800):
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()


def test_pack_one_matches_default_single(monkeypatch):
    texts = synth.corpus(2000, V=8000, len_min=30, len_max=70)
    monkeypatch.setenv("TFIDF_PACK_DOCS", "1")
    a = ShardIndex()
    a.add_documents(texts)
    a.commit()
    monkeypatch.setenv("TFIDF_PACK_DOCS", "7")
    b = ShardIndex()
    b.add_documents(texts)
    b.commit()
    sa, sb = a.stats(), b.stats()
    assert sa["pack_docs"] == 1 and sb["pack_docs"] == 7
    for k in ("doc_count", "sum_ttf", "num_terms", "nnz"):
        assert sa[k] == sb[k]
    for d in range(0, 2000, 37):
        assert a.doc_terms(d) == b.doc_terms(d)
    for q in synth.queries(20, lo=1, hi=3000):
        assert a.search(q, 10) == b.search(q, 10)
    a.close()
    b.close()
