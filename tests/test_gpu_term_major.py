"""GPU parity of the term-major inversion (TFIDF_INVERSION_TERM, kernels_term.hip):
the layout AUTO picks for huge vocabularies (SURVEY §8 cfg 5), forced here at
test sizes.  Same bar as test_gpu_parity.py: TF/DF/stats and hit lists
bit-exact against the oracle, scores as float32 bit patterns; the block-major
build of the same corpus must agree bit for bit as well.
"""
import random

import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd import _lib as L
from tfidf_amd.engine import ShardIndex

from test_gpu_parity import assert_hits_equal

pytestmark = pytest.mark.gpu


def build(texts, inversion, cap_log2=18, keys=None):
    g = ShardIndex(vocab_capacity_log2=cap_log2, inversion=inversion)
    g.add_documents(texts, keys)
    g.commit()
    return g


def oracle_of(texts, keys=None):
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(keys[i] if keys else str(i).encode(), t)
    o.commit()
    return o


def test_fixture_term_major(lucene_fixture):
    texts = [d["text"].encode() for d in lucene_fixture["docs"]]
    keys = [d["name"].encode() for d in lucene_fixture["docs"]]
    g = build(texts, L.INVERSION_TERM, keys=keys)
    o = oracle_of(texts, keys)
    f = lucene_fixture
    s = g.stats()
    assert s["doc_count"] == f["field_stats"]["docCount"]
    assert s["sum_ttf"] == f["field_stats"]["sumTotalTermFreq"]
    assert s["nnz"] == f["field_stats"]["sumDocFreq"]
    for t in f["terms"]:
        assert g.df(t["term"].encode())[0] == t["df"]
    for q in [b"fast food", b"cat", b"best wireless earbuds", b"at night", b"nothing-here"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
        assert_hits_equal(g.search(q, 3), o.search(q, 3))
    g.close()
    o.close()


@pytest.fixture(scope="module")
def multi_block():
    # > 2 doc blocks of 8192, so segments start mid-list and end mid-list
    texts = synth.corpus(20000, V=30000, len_min=20, len_max=90)
    o = oracle_of(texts)
    t = build(texts, L.INVERSION_TERM)
    b = build(texts, L.INVERSION_BLOCK)
    yield t, b, o, texts
    t.close()
    b.close()
    o.close()


def test_multi_block_stats_and_df(multi_block):
    t, b, o, _ = multi_block
    st = t.stats()
    assert st["term_major"] == 1 and b.stats()["term_major"] == 0
    assert (st["doc_count"], st["sum_ttf"], st["num_terms"], st["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    vocab = o.vocab()
    rng = random.Random(5)
    for w in rng.sample(sorted(vocab), 300) + [synth.word(1), synth.word(2)]:
        assert t.df(w)[0] == vocab.get(w, 0) == b.df(w)[0]


def test_multi_block_queries(multi_block):
    t, b, o, _ = multi_block
    qs = synth.queries(20, lo=1, hi=3000) + [b"aaaa", b"aaaa aaab aaac aaad aaae aaaf", b"zzzzzz"]
    for q in qs:
        want = o.search(q, 0)
        assert_hits_equal(t.search(q, 0), want)
        assert_hits_equal(b.search(q, 0), want)
        assert_hits_equal(t.search(q, 10), o.search(q, 10))
    for k in (10, 100):
        d1, s1, c1 = t.search_batch(qs, k)
        for i, q in enumerate(qs):
            got = list(zip(d1[i, :c1[i]].tolist(), s1[i, :c1[i]].tolist()))
            assert_hits_equal(got, o.search(q, k))


def test_large_vocab_short_docs():
    """cfg-5 shape at test size: Zipf over a 5 M-term vocabulary, 48-80
    tokens per doc, a 2^22-slot dictionary (mostly empty slots)."""
    texts = synth.corpus(12000, V=5_000_000, len_min=48, len_max=80)
    o = oracle_of(texts)
    g = build(texts, L.INVERSION_AUTO, cap_log2=22)      # > 2^21 slots: AUTO picks term-major
    st = g.stats()
    assert st["term_major"] == 1
    assert (st["doc_count"], st["sum_ttf"], st["num_terms"], st["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in range(0, 12000, 397):
        assert g.doc_terms(d) == o.doc_terms(d)
    for q in synth.queries(15, lo=1, hi=20000) + synth.queries(5, lo=100000, hi=4_000_000, seed=9):
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
        assert_hits_equal(g.search(q, 100), o.search(q, 100))
    g.close()
    o.close()


def test_term_major_long_docs_and_updates():
    rng = random.Random(13)
    cdf = synth.zipf_cdf(20000)
    texts = synth.corpus(300, V=20000, len_min=10, len_max=300)
    for n in (1500, 30000):
        ranks = synth.doc_ranks(7, n, n, n, cdf)
        texts.insert(rng.randrange(len(texts)), b" ".join(synth.word(int(r)) for r in ranks))
    keys = [b"k%d" % (i % 250) for i in range(len(texts))]     # repeated keys replace earlier docs
    g = build(texts, L.INVERSION_TERM, keys=keys)
    o = oracle_of(texts, keys)
    assert g.stats()["num_docs"] == o.num_docs
    for q in synth.queries(10, lo=1, hi=2000):
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()


def test_term_major_empty():
    g = build([b"", b" .. "], L.INVERSION_TERM)
    assert g.stats()["doc_count"] == 0
    assert g.search(b"anything", 0) == []
    g.close()


@pytest.mark.parametrize("inversion", [L.INVERSION_BLOCK, L.INVERSION_TERM])
def test_large_tf_escapes(monkeypatch, inversion):
    """Term frequencies the packed fields cannot hold take the escape lists:
    block-major postings hold tf < 2047 (a term 3 000 times in one document
    escapes); the term-major sort words are squeezed to 4 tf bits here
    (TFIDF_TEST_TERM_TF_BITS), so every tf >= 15 escapes.  Counts, DF and
    scores must still equal the oracle's."""
    monkeypatch.setenv("TFIDF_TEST_TERM_TF_BITS", "4")
    rng = random.Random(5)
    texts = []
    for i in range(300):
        words = [rng.choice([b"alpha", b"beta", b"gamma", b"delta", b"eps%d" % (i % 7)]) for _ in range(rng.randint(5, 60))]
        if i % 50 == 3:
            words += [b"alpha"] * 3000 + [b"gamma"] * 40
        rng.shuffle(words)
        texts.append(b" ".join(words))
    g = build(texts, inversion)
    o = oracle_of(texts)
    s = g.stats()
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in range(len(texts)):
        assert g.doc_terms(d) == o.doc_terms(d), d
    for q in [b"alpha", b"gamma", b"alpha beta", b"eps3 gamma", b"alpha AND gamma"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
        assert_hits_equal(g.search(q, 10), o.search(q, 10))
    g.close()
    o.close()


@pytest.mark.parametrize("n_docs", [8, 40, 100])
def test_small_shards_tf_field(n_docs):
    # few documents leave 56 - slot - doc bits >= 32 for tf: the field is
    # capped at 24 bits (a 32-bit shift made every tf an escape and the host
    # divided by zero at 33..64 documents: the bench's 40-book CPU sample)
    rng = random.Random(n_docs)
    texts = [b" ".join([b"alpha"] * rng.randint(1, 300) + [synth.word(rng.randint(1, 500)) for _ in range(200)])
             for _ in range(n_docs)]
    g = build(texts, L.INVERSION_TERM)
    o = oracle_of(texts)
    assert g.stats()["term_major"] == 1
    for d in range(n_docs):
        assert g.doc_terms(d) == o.doc_terms(d)
    for q in [b"alpha", b"alpha aaab", b"aaac aaad aaae"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
        assert_hits_equal(g.search(q, 5), o.search(q, 5))
    g.close()
    o.close()
