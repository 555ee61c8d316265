"""Pin the CPU oracle against the reference's committed Lucene 9.8.0 index.

The golden fixture (tests/golden/lucene_sample8.json) is decoded from
TF-IDF-System-Core/src/main/resources/documents/.luceneIndex by
tests/golden/make_lucene_fixture.py.  It pins tokenisation, per-(doc, term)
TF, DF, norm bytes, docCount, sumTotalTermFreq and sumDocFreq.  Scores are
not pinned by any reference artefact; the BM25 expectations below are the
survey's independent NumPy derivation and a float32
restatement in this file — flagged "parity unpinned" in DESIGN.md.
"""
import numpy as np
import pytest

from oracle import oracle as O


@pytest.fixture(scope="module")
def ix(lucene_fixture):
    o = O.OracleIndex()
    for d in lucene_fixture["docs"]:
        o.add_doc(d["name"].encode(), d["text"].encode())
    o.commit()
    yield o
    o.close()


def test_field_stats(ix, lucene_fixture):
    fs = lucene_fixture["field_stats"]
    assert ix.doc_count == fs["docCount"] == 8
    assert ix.sum_ttf == fs["sumTotalTermFreq"] == 252
    assert ix.num_terms == fs["numTerms"] == 13
    assert sum(ix.df(t["term"].encode()) for t in lucene_fixture["terms"]) == fs["sumDocFreq"]


def test_norm_bytes(ix, lucene_fixture):
    norms = lucene_fixture["norms"]
    assert [ix.doc_norm(d) for d in range(8)] == norms[:8]
    # docs 8..20 of the committed segment had no tokens -> norm 0 (IndexingChain)
    assert all(n == 0 for n in norms[8:])
    assert O.int_to_byte4(0) == 0


def test_doc_lengths(ix, lucene_fixture):
    assert [ix.doc_len(d) for d in range(8)] == lucene_fixture["doc_lengths_from_postings"][:8]


def test_postings_tf_df(ix, lucene_fixture):
    vocab = ix.vocab()
    assert set(vocab) == {t["term"].encode() for t in lucene_fixture["terms"]}
    for t in lucene_fixture["terms"]:
        term = t["term"].encode()
        assert ix.df(term) == t["df"]
        for doc, tf in t["postings"]:
            assert ix.doc_terms(doc)[term] == tf
    # and nothing else: every doc's term set equals the fixture's
    per_doc = {}
    for t in lucene_fixture["terms"]:
        for doc, tf in t["postings"]:
            per_doc.setdefault(doc, {})[t["term"].encode()] = tf
    for d in range(8):
        assert ix.doc_terms(d) == per_doc.get(d, {})


@pytest.mark.parametrize("n,byte,decoded", [
    (12, 0x0C, 12), (18, 0x12, 18), (24, 0x18, 24), (28, 0x1C, 28),
    (38, 0x26, 38), (50, 0x2D, 50), (58, 0x30, 56), (0, 0, 0), (1, 1, 1), (23, 23, 23),
])
def test_smallfloat_known_answers(n, byte, decoded):
    assert O.int_to_byte4(n) == byte
    assert O.byte4_to_int(byte) == decoded


def test_smallfloat_monotone_roundtrip():
    prev = -1
    for b in range(256):
        v = O.byte4_to_int(b)
        assert v > prev
        assert O.int_to_byte4(v) == b
        prev = v
    assert O.byte4_to_int(255) == 2 ** 31 - 1 or O.byte4_to_int(255) > 2 ** 30


# derived (NOT Lucene-executed) BM25 worker outputs.
DERIVED = {
    b"fast food": [("file6.txt", 0.592446506023407), ("file8.txt", 0.590718150138855),
                   ("file7.txt", 0.5865983366966248), ("file5.txt", 0.5780282616615295),
                   ("file.txt", 0.5766979455947876), ("file3.txt", 0.5500096678733826)],
    b"cat": [("file2.txt", 0.5909903049468994), ("file3.txt", 0.4471917152404785),
             ("file5.txt", 0.40945401787757874), ("file4.txt", 0.3554600477218628)],
    b"best wireless earbuds": [("file4.txt", 2.0121634006500244), ("file7.txt", 1.1737618446350098),
                               ("file5.txt", 0.9769635200500488), ("file6.txt", 0.6981337666511536)],
    b"kheder": [("file3.txt", 0.2667396664619446), ("file.txt", 0.19808320701122284),
                ("file8.txt", 0.17936666309833527), ("file6.txt", 0.16388176381587982),
                ("file7.txt", 0.16388176381587982), ("file5.txt", 0.1364045888185501)],
    b"at night": [("file2.txt", 1.1819806098937988), ("file3.txt", 0.894383430480957),
                  ("file5.txt", 0.8189080357551575), ("file4.txt", 0.7109200954437256)],
}


@pytest.mark.parametrize("q", list(DERIVED))
def test_bm25_matches_survey_derivation(ix, q):
    got = [(ix.doc_key(d).decode(), s) for d, s in ix.search(q)]
    assert [n for n, _ in got] == [n for n, _ in DERIVED[q]]
    for (_, a), (_, b) in zip(got, DERIVED[q]):
        assert np.float32(a) == np.float32(b)          # bit-exact as float32


def test_tie_break_doc_ascending(ix):
    hits = ix.search(b"kheder")
    # file6 (doc 5) and file7 (doc 6) tie exactly -> lower docID first
    assert hits[3][1] == hits[4][1] and hits[3][0] == 5 and hits[4][0] == 6


def _np_bm25_scores(ix, terms_boosts):
    """Independent float32 NumPy restatement of BM25Similarity 9.8.0."""
    N = ix.doc_count
    avg = np.float32(ix.sum_ttf / float(N))
    L = np.array([O.byte4_to_int(i) for i in range(256)], np.float32)
    k1, b = np.float32(1.2), np.float32(0.75)
    cache = np.float32(1) / (k1 * ((np.float32(1) - b) + b * L / avg))
    acc = {}
    for term, boost in terms_boosts:
        df = ix.df(term)
        if df == 0:
            continue
        idf = np.float32(np.log(1.0 + (N - df + 0.5) / (df + 0.5)))
        w = np.float32(boost) * idf
        for d in range(ix.num_docs):
            tf = ix.doc_terms(d).get(term)
            if tf is None:
                continue
            s = w - w / (np.float32(1) + np.float32(tf) * cache[ix.doc_norm(d)])
            acc[d] = acc.get(d, 0.0) + float(np.float32(s))
    hits = sorted(((np.float32(v), d) for d, v in acc.items()), key=lambda x: (-x[0], x[1]))
    return [(d, float(s)) for s, d in hits]


@pytest.mark.parametrize("q", [b"fast food", b"fast fast food", b"kheder helo 2024", b"night at night",
                               b"wireless best earbuds cat", b"zzz"])
def test_bm25_numpy_restatement(ix, q):
    want = _np_bm25_scores(ix, O.query_terms(q))
    assert ix.search(q) == want


def test_empty_query_is_parse_exception(ix):
    # QueryParser.parse("") throws ParseException (Encountered <EOF>); Worker answers []
    for q in (b"", b"  \t "):
        with pytest.raises(O.QuerySyntaxError):
            ix.search(q)


def test_duplicate_query_terms_boost():
    assert O.query_terms(b"fast Fast food fast") == [(b"fast", 3.0), (b"food", 1.0)]


def test_operator_words_parse(ix):
    # escape() leaves AND / OR / NOT: they stay operators (tests/test_query_operators.py)
    assert {d for d, _ in ix.search(b"fast AND food")} == {d for d, _ in ix.search(b"fast")}
    assert ix.search(b"NOT cat") == []
    assert ix.search(b"cat OR night") == ix.search(b"cat night")


def test_escaped_specials_are_plain_text(ix):
    # QueryParser.escape turns "+fast -food (cat)" into literal text
    assert ix.search(b"+fast -food (cat)") == ix.search(b"fast food cat")


def test_topk_prefix_of_all_hits(ix):
    full = ix.search(b"fast food cat at")
    for k in (1, 3, 5, 50):
        assert ix.search(b"fast food cat at", k=k) == full[:k]


def test_leader_merge_sum_and_name_order():
    w1 = [(b"file6.txt", 0.5), (b"b.txt", 0.25)]
    w2 = [(b"a.txt", 1.0), (b"file6.txt", 0.125)]
    assert O.leader_merge([w1, w2]) == [(b"a.txt", 1.0), (b"b.txt", 0.25), (b"file6.txt", 0.625)]
    assert O.leader_merge([]) == []


def test_update_document_replaces_by_key():
    o = O.OracleIndex()
    o.add_doc(b"a", b"fast food")
    o.add_doc(b"b", b"cat")
    o.add_doc(b"a", b"night")      # updateDocument(Term("path","a"))
    o.commit()
    assert o.num_docs == 2
    assert [o.doc_key(d) for d in range(2)] == [b"b", b"a"]
    assert o.df(b"fast") == 0 and o.df(b"night") == 1
    o.close()
