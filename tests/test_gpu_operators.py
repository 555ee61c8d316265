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
