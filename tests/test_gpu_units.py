"""GPU parity of the batched top-k path by query units (k_score_units:
workgroup per (query, doc-block range), dense block accumulator, running k-th
key filter) against the CPU oracle.

The unit path runs for batches with k <= 64 of plain disjunctions over the
block-major layout once the batch has num_cus * 16 (query, block) pairs; the
corpora here have several 8192-document blocks so that hits, ties and top-k
lists cross blocks and waves.  TFIDF_UNIT_POST forces queries to be split
into several block ranges (the merge of several units of one query).
Bar: doc ids and float32 score bits identical to the oracle.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

pytestmark = pytest.mark.gpu


def f32bits(x):
    return np.float32(x).view(np.int32).item()


def rows(docs, scores, counts, i):
    return list(zip(docs[i, :counts[i]].tolist(), [f32bits(s) for s in scores[i, :counts[i]].tolist()]))


def want(o, q, k):
    try:
        return [(d, f32bits(s)) for d, s in o.search(q, k)]
    except O.QuerySyntaxError:      # the reference answers [] (Worker.java:182-185); a batch row is empty
        return []


@pytest.fixture(scope="module")
def corpus():
    # 3 blocks of Zipf text + a block of tie-storm documents (equal scores
    # across blocks and waves: the doc-ascending tie order is exercised)
    texts = synth.corpus(26_000, V=6_000, len_min=20, len_max=120)
    texts += [b"tie storm words here"] * 6_000 + [b"tie storm"] * 1_000
    g = ShardIndex(vocab_capacity_log2=16)
    g.add_documents(texts)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    yield g, o
    g.close()
    o.close()


def queries():
    qs = synth.queries(1500, lo=1, hi=3000)
    qs += synth.queries(200, n_terms=1, lo=1, hi=200)                  # dense single terms
    qs += [b"tie", b"tie storm", b"storm words aaaa", b"zzzzzz", b"", b"... !!",
           b"aaaa aaaa aaab", b"qqqqqq aaaa", b" ".join(synth.word(r) for r in range(1, 60))]
    return qs


# TFIDF_WUNIT_LIGHT = postings per block up to which a query takes the wave
# units (k_score_wunits); above it the workgroup units (k_score_units).  0:
# every query on workgroup units; 10^9: every query on wave units (blocks of
# more than 700 postings then take the 16-pass sub-range path).
@pytest.mark.parametrize("light", [None, "0", "1000000000"])
@pytest.mark.parametrize("k", [1, 10, 64])
def test_units_match_oracle(corpus, k, light, monkeypatch):
    g, o = corpus
    if light is not None:
        monkeypatch.setenv("TFIDF_WUNIT_LIGHT", light)
    qs = queries()
    before = g.stats()["unit_batches"]
    docs, scores, counts = g.search_batch(qs, k)
    assert g.stats()["unit_batches"] == before + 1           # the unit path ran
    for i, q in enumerate(qs):
        assert rows(docs, scores, counts, i) == want(o, q, k), q


@pytest.mark.parametrize("light", ["0", "1000000000"])
def test_units_split_queries(corpus, monkeypatch, light):
    g, o = corpus
    qs = queries()
    monkeypatch.setenv("TFIDF_WUNIT_LIGHT", light)
    monkeypatch.setenv("TFIDF_UNIT_POST", "60")              # most queries cut into several block ranges
    s0 = g.stats()
    docs, scores, counts = g.search_batch(qs, 10)
    s1 = g.stats()
    assert s1["unit_batches"] == s0["unit_batches"] + 1
    assert s1["unit_count"] - s0["unit_count"] > len(qs) * 2
    for i, q in enumerate(qs):
        assert rows(docs, scores, counts, i) == want(o, q, 10), q


def test_units_same_as_other_paths(corpus, monkeypatch):
    g, _ = corpus
    qs = queries()
    d1, s1, c1 = g.search_batch(qs, 10)
    monkeypatch.setenv("TFIDF_NO_UNITS", "1")
    d2, s2, c2 = g.search_batch(qs, 10)
    for i in range(len(qs)):
        assert rows(d1, s1, c1, i) == rows(d2, s2, c2, i)
    for i in range(0, len(qs), 37):
        got = [(d, f32bits(s)) for d, s in g.search(qs[i], 10)]
        assert rows(d1, s1, c1, i) == got


def test_units_not_for_large_k_or_long_queries(corpus):
    g, o = corpus
    qs = queries()
    before = g.stats()["unit_batches"]
    docs, scores, counts = g.search_batch(qs, 65)            # k > 64: wave-per-pair path
    assert g.stats()["unit_batches"] == before
    for i in range(0, len(qs), 11):
        assert rows(docs, scores, counts, i) == want(o, qs[i], 65)
    long_q = qs[:-1] + [b" ".join(synth.word(r) for r in range(1, 80))]   # a query of > 64 terms
    docs, scores, counts = g.search_batch(long_q, 10)
    assert g.stats()["unit_batches"] == before
    assert rows(docs, scores, counts, len(long_q) - 1) == want(o, long_q[-1], 10)


def test_query_timing_toggle(corpus):
    # serving configuration: no HIP events around searches (tfidf_set_query_timing)
    g, o = corpus
    qs = queries()[:50]
    g.set_query_timing(False)
    try:
        off = [g.search(q, 10) for q in qs[:20]]
        assert g.last_search_ms() == (-1.0, -1.0)
        d_off, s_off, c_off = g.search_batch(qs, 10)
    finally:
        g.set_query_timing(True)
    on = [g.search(q, 10) for q in qs[:20]]
    assert g.last_search_ms()[1] > 0
    d_on, s_on, c_on = g.search_batch(qs, 10)
    assert off == on
    assert (c_off == c_on).all() and (d_off == d_on).all() and (s_off.view("i4") == s_on.view("i4")).all()


@pytest.mark.parametrize("chunks", ["1", "3", "7"])
def test_pipelined_batch_chunks_equal_oracle(corpus, chunks, monkeypatch):
    """tfidf_search_batch prepares chunk c + 1 on the host while chunk c scores:
    any chunking (uneven chunks, a chunk whose queries have no present term)
    gives the oracle's rows in the caller's order."""
    g, o = corpus
    qs = queries()[:1200] + [b"zzzzzz qqqqqq"] * 300 + queries()[1200:]
    monkeypatch.setenv("TFIDF_BATCH_CHUNKS", chunks)
    docs, scores, counts = g.search_batch(qs, 10)
    for i in range(0, len(qs), 7):
        assert rows(docs, scores, counts, i) == want(o, qs[i], 10), (chunks, i, qs[i])
    assert all(counts[i] == 0 for i in range(1200, 1500))
