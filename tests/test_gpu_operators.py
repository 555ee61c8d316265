"""GPU parity for the operator words AND / OR / NOT (Worker.java:225-227:
QueryParser.escape leaves them, so Lucene answers conjunctions and exclusions).
The HIP scorer (k_score_blocks<true>, and k_score_pairs handing operator
queries over in batches) against the C oracle, which tests/test_query_operators.py
holds equal to an independent Python restatement.  Bar: doc ids and float32
score bits identical.
"""
import random

import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd._lib import INVERSION_TERM, QuerySyntaxError
from tfidf_amd.engine import ShardIndex
from test_gpu_parity import assert_hits_equal, build_pair
from test_query_operators import FIX_QUERIES

pytestmark = pytest.mark.gpu


def both(g, o, q, k):
    try:
        want = o.search(q, k)
    except O.QuerySyntaxError:
        with pytest.raises(QuerySyntaxError):
            g.search(q, k)
        return None
    got = g.search(q, k)
    assert_hits_equal(got, want)
    return want


def batch_equal(g, o, qs, k):
    docs, scores, counts = g.search_batch(qs, k)
    for i, q in enumerate(qs):
        try:
            want = o.search(q, k)
        except O.QuerySyntaxError:
            want = []                                  # a query that does not parse has no hits
        got = list(zip(docs[i, :counts[i]].tolist(), scores[i, :counts[i]].tolist()))
        assert_hits_equal(got, want)


@pytest.fixture(scope="module")
def fx(lucene_fixture):
    texts = [d["text"].encode() for d in lucene_fixture["docs"]]
    keys = [d["name"].encode() for d in lucene_fixture["docs"]]
    g, o = build_pair(texts, keys)
    yield g, o
    g.close()
    o.close()


@pytest.mark.parametrize("k", [0, 1, 3, 10])
def test_fixture_operator_queries(fx, k):
    g, o = fx
    for q in FIX_QUERIES + [b"fast AND", b"OR fast", b""]:
        both(g, o, q, k)


def test_fixture_operator_batch(fx):
    g, o = fx
    batch_equal(g, o, FIX_QUERIES + [b"fast AND", b"NOT NOT x", b"fast food"], 10)


def op_queries(n, seed, lo=30, hi=3000):
    """Random operator queries over mid-frequency synthetic words."""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        parts = []
        for i in range(rng.randint(1, 5)):
            if i and rng.random() < 0.45:
                parts.append(rng.choice([b"AND", b"OR", b"AND"]))
            if rng.random() < 0.2:
                parts.append(b"NOT")
            w = synth.word(rng.randint(lo, hi))
            if rng.random() < 0.15:
                w += b"-" + synth.word(rng.randint(1, hi))
            parts.append(w)
        out.append(b" ".join(parts))
    return out


@pytest.fixture(scope="module", params=["block", "term"])
def zipf(request):
    texts = synth.corpus(20000, V=20000, len_min=30, len_max=220)
    if request.param == "term":
        g = ShardIndex(inversion=INVERSION_TERM)
        g.add_documents(texts)
        g.commit()
        o = O.OracleIndex()
        for i, t in enumerate(texts):
            o.add_doc(str(i).encode(), t)
        o.commit()
    else:
        g, o = build_pair(texts)
    yield g, o
    g.close()
    o.close()


def test_zipf_operator_single(zipf):
    g, o = zipf
    for q in op_queries(60, 5) + [b"aaaa AND aaab", b"aaaa NOT aaab", b"aaab AND aaac AND aaad AND aaae"]:
        for k in (0, 10, 100):
            both(g, o, q, k)


def test_zipf_operator_batch_mixed(zipf):
    # 2000 queries x 3 blocks >= 16 pairs per CU: the wave-per-pair kernel runs
    # and hands operator queries (and heavy plain pairs) to k_score_blocks
    g, o = zipf
    plain = synth.queries(1000, lo=20, hi=4000)
    ops = op_queries(1000, 9)
    qs = [x for pair in zip(plain, ops) for x in pair]
    for k in (10, 100):
        batch_equal(g, o, qs, k)


@pytest.mark.parametrize("cap", [None, 3])
def test_concurrent_searches_coalesce_into_batches(monkeypatch, cap):
    """Concurrent single searches from many threads (the reference's request
    threads, Worker.java:175-186) share batched scoring launches and each get
    exactly tfidf_search's answer, including syntax errors.  cap = 3: batches
    of at most 3 requests (TFIDF_COALESCE_MAX), so a leader's own request is
    often left over (it leads again) and left-over requests need a new leader."""
    import threading
    if cap:
        monkeypatch.setenv("TFIDF_COALESCE_MAX", str(cap))
    texts = synth.corpus(6000, V=3000, len_min=10, len_max=120)
    g = ShardIndex()
    g.add_documents(texts)
    g.commit()
    qs = synth.queries(400, lo=1, hi=2500) + [b"alpha AND beta", b"fast AND", b"aaaa NOT aaab"]
    want = {}
    for q in qs:
        try:
            want[q] = g.search(q, 10)
        except QuerySyntaxError:
            want[q] = "syntax"
    got, errs = {}, []

    def worker(part):
        for q in part:
            try:
                got[q] = g.search_coalesced(q, 10, wait_us=200)
            except QuerySyntaxError:
                got[q] = "syntax"
            except Exception as e:                      # noqa: BLE001
                errs.append(e)

    ths = [threading.Thread(target=worker, args=(qs[i::16],)) for i in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs
    for q in qs:
        if want[q] == "syntax":
            assert got[q] == "syntax", q
        else:
            assert_hits_equal(got[q], want[q])
    st = g.stats()
    assert st["coalesced_queries"] == len(qs)
    assert st["coalesced_batches"] < len(qs)             # some searches shared a launch
    if cap:
        # every batch holds 1..cap requests: a waiter whose request a running
        # leader took never leads an (empty) batch of its own
        assert len(qs) / cap <= st["coalesced_batches"] <= st["coalesced_queries"]
    g.close()
