"""BASELINE cfg 1 — the reference's own workload: "leader + 1 worker over a
few hundred plain-text books, 3-term query, top-10 ranking".  Books are not
available offline, so the stand-in is SURVEY §8(d)'s: 300 documents x U[80 k,
120 k] tokens of the Zipf corpus (~150 MB).  Book-sized documents take the
chunk-parallel path (k_tokenize_chunk + k_long_rows); these tests hold it to
the CPU oracle, including chunk boundaries inside tokens and joiner runs.
"""
import os
import random

import numpy as np
import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex
from test_gpu_parity import assert_hits_equal, build_pair, random_text

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def books(tmp_path_factory):
    dc = synth.DeviceCorpus(300, V=100_000, len_min=80_000, len_max=120_000, seed=synth.SEED + 11)
    text, offs = dc.to_host()
    dc.free()
    raw = text.tobytes()
    texts = [raw[int(offs[i]):int(offs[i + 1])] for i in range(300)]
    names = [b"book%03d.txt" % i for i in range(300)]
    o = O.OracleIndex()
    for n, t in zip(names, texts):
        o.add_doc(n, t)
    o.commit()
    d = tmp_path_factory.mktemp("books")
    docs = d / "documents"
    docs.mkdir()
    for n, t in zip(names, texts):
        (docs / n.decode()).write_bytes(t)
    yield texts, names, o, str(docs)
    o.close()


def test_books_index_equals_oracle(books):
    texts, names, o, _ = books
    g = ShardIndex()
    g.add_documents(texts, names)
    g.commit()
    s = g.stats()
    assert s["long_docs"] == 300 and s["long_chunked"] == 300      # every book took the chunk path
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in (0, 1, 77, 150, 299):
        assert g.doc_terms(d) == o.doc_terms(d), d
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))
    for q in synth.queries(20, lo=100, hi=10_000) + [b"aaaa", b"aaaa AND aaab NOT aaac"]:
        assert_hits_equal(g.search(q, 10), o.search(q, 10))
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()


@pytest.mark.parametrize("cap_log2,inversion", [(22, "auto"), (18, "block")])
def test_books_many_groups_wide_dictionary(books, monkeypatch, cap_log2, inversion):
    """The chunk path in many groups (TFIDF_TEST_PAIR_UNITS: ~15 books per
    group instead of one group for all) and with bucketed pair lists of two
    windows per bucket (2^22 dictionary slots: 64 buckets of 2^16 slots), or
    with block-major CSR rows (8 dictionary ranges: range splits at window ends)."""
    from tfidf_amd import _lib as L
    texts, names, o, _ = books
    monkeypatch.setenv("TFIDF_TEST_PAIR_UNITS", "5000")
    inv = L.INVERSION_BLOCK if inversion == "block" else L.INVERSION_AUTO
    g = ShardIndex(vocab_capacity_log2=cap_log2, inversion=inv)
    g.add_documents(texts, names)
    g.commit()
    s = g.stats()
    assert s["long_chunked"] == 300
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in (0, 14, 15, 16, 150, 299):                         # group edges (~15 books per group)
        assert g.doc_terms(d) == o.doc_terms(d), d
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))
    for q in synth.queries(8, lo=100, hi=10_000, seed=7) + [b"aaaa"]:
        assert_hits_equal(g.search(q, 10), o.search(q, 10))
    g.close()


def test_books_leader_one_worker(books):
    """Leader + 1 worker (Leader.java:39-92 over Worker.java:57-94,222-241):
    the worker's JSON hits and the leader's name-ordered map equal the oracle."""
    from tfidf_amd.reference_api import Leader, Worker
    texts, names, o, docs = books
    w = Worker(docs, os.path.join(docs, ".luceneIndex"))
    w.init()
    for q in synth.queries(5, lo=100, hi=10_000, seed=99):
        got = w.process_documents(q.decode())
        want = o.search(q)
        assert [r["document"]["name"].encode() for r in got] == [o.doc_key(dd) for dd, _ in want]
        assert [np.float32(r["score"]) for r in got] == [np.float32(sc) for _, sc in want]
        top = Leader([w]).start(q.decode())
        assert list(top) == sorted(top)
        assert {k.encode(): v for k, v in top.items()} == {o.doc_key(dd): float(np.float32(sc)) for dd, sc in want}
    w.close()


def test_chunk_boundaries_punctuation_books():
    """Long documents of joiner-heavy text (: . ' , ; _ runs, digits, tabs) and
    long words straddling the 2 KB chunk cores.  Documents holding a token of
    more than 255 characters (runs of joined pieces, and one deliberate
    300-char word) go to k_tokenize_long as a whole; the others take the
    chunk path — every document must equal the oracle either way."""
    rng = random.Random(2024)
    texts = []
    for i in range(24):
        parts = []
        while sum(len(x) for x in parts) < rng.randint(20_000, 60_000):
            r = rng.random()
            if r < 0.7:
                parts.append(random_text(rng, rng.randint(1, 400)) + b" ")
            elif r < 0.9:
                parts.append(b"".join(rng.choice([b"ab", b"C9", b"x_", b"a.b", b"3,1", b"d'e"]) for _ in range(rng.randint(1, 60))) + b" ")
            else:
                parts.append(b" " + b"w" * rng.randint(9, 250) + b" ")
        texts.append(b"".join(parts))
    texts[5] = texts[5][:3000] + b" " + b"q" * 300 + b" " + texts[5][3000:]
    g, o = build_pair(texts)
    s = g.stats()
    assert s["long_docs"] == 24 and 1 <= s["long_chunked"] <= 23     # doc 5 (300-char word) falls back
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in range(len(texts)):
        assert g.doc_terms(d) == o.doc_terms(d), d
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))
    for q in [b"ab", b"c9 x_", b"a.b 3,1", b"w" * 12, b"d'e"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()
