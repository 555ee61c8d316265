"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle and
the golden fixture decoded from the reference's Lucene 9.8.0 index.

Bar: TF, DF, norms, doc lengths, docCount, sumTotalTermFreq, hit sets and
top-k doc ids bit-exact; scores compared as float32 bit patterns (the engine
reproduces Lucene's float operation order, so the tolerance is zero; the
north_star tolerance for fp32 would be 1e-4 relative).
"""
import os
import random

import numpy as np
import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex
from tfidf_amd._lib import QuerySyntaxError, UnsupportedInput

pytestmark = pytest.mark.gpu


def f32bits(x):
    return np.float32(x).view(np.int32).item()


def assert_hits_equal(got, want):
    assert [d for d, _ in got] == [d for d, _ in want]
    assert [f32bits(s) for _, s in got] == [f32bits(s) for _, s in want]


QUERY_COUNTERS = ("coalesced_batches", "coalesced_queries", "unit_batches", "unit_count", "fused_queries")


def index_stats(g):
    """tfidf_stats without the lifetime query counters (they grow with searches)."""
    return {k: v for k, v in g.stats().items() if k not in QUERY_COUNTERS}


def build_pair(texts, keys=None, cap_log2=18):
    g = ShardIndex(vocab_capacity_log2=cap_log2)
    g.add_documents(texts, keys)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(keys[i] if keys else str(i).encode(), t)
    o.commit()
    return g, o


# ---------------------------------------------------------------------------
# golden fixture (reference's committed Lucene index)

@pytest.fixture(scope="module")
def fx(lucene_fixture):
    texts = [d["text"].encode() for d in lucene_fixture["docs"]]
    keys = [d["name"].encode() for d in lucene_fixture["docs"]]
    g, o = build_pair(texts, keys)
    yield g, o, lucene_fixture
    g.close()
    o.close()


def test_fixture_collection_stats(fx):
    g, _, f = fx
    s = g.stats()
    assert s["doc_count"] == f["field_stats"]["docCount"] == 8
    assert s["sum_ttf"] == f["field_stats"]["sumTotalTermFreq"] == 252
    assert s["num_terms"] == f["field_stats"]["numTerms"] == 13
    assert s["nnz"] == f["field_stats"]["sumDocFreq"] == 58
    assert s["num_docs"] == 8


def test_fixture_tf_df_norms(fx):
    g, _, f = fx
    per_doc = {}
    for t in f["terms"]:
        assert g.df(t["term"].encode())[0] == t["df"]
        for d, tf in t["postings"]:
            per_doc.setdefault(d, {})[t["term"].encode()] = tf
    for d in range(8):
        assert g.doc_terms(d) == per_doc[d]
        ln, nm = g.doc_len(d)
        assert ln == f["doc_lengths_from_postings"][d]
        assert nm == f["norms"][d]


@pytest.mark.parametrize("q", [b"fast food", b"cat", b"best wireless earbuds", b"kheder", b"at night",
                               b"fast fast food", b"FAST Food!", b"2024 helo", b"nothing here",
                               b"+fast -(food)", b"e-mail kheder:helo"])
def test_fixture_search_all_hits(fx, q):
    g, o, _ = fx
    assert_hits_equal(g.search(q, k=0), o.search(q, k=0))


@pytest.mark.parametrize("k", [1, 3, 5, 100])
def test_fixture_search_topk(fx, k):
    g, o, _ = fx
    for q in [b"fast food", b"kheder", b"cat at night causes"]:
        assert_hits_equal(g.search(q, k=k), o.search(q, k=k))


def test_operator_words_are_operators(fx):
    # the operator-word parity suite is tests/test_gpu_operators.py
    g, o, _ = fx
    assert_hits_equal(g.search(b"fast AND food", 0), o.search(b"fast AND food", 0))
    with pytest.raises(QuerySyntaxError):
        g.search(b"")


def test_reference_worker_and_leader(tmp_path, lucene_fixture):
    from tfidf_amd.reference_api import Leader, Worker
    docs = tmp_path / "documents"
    docs.mkdir()
    for d in lucene_fixture["docs"]:
        (docs / d["name"]).write_bytes(d["text"].encode())
    w = Worker(str(docs), str(docs / ".luceneIndex"))
    w.init()
    o = O.OracleIndex()
    for d in sorted(lucene_fixture["docs"], key=lambda d: d["name"]):
        o.add_doc(d["name"].encode(), d["text"].encode())
    o.commit()
    for q in ["fast food", "kheder", "best wireless earbuds"]:
        got = w.process_documents(q)
        want = [{"document": {"name": o.doc_key(d).decode()}, "score": s} for d, s in o.search(q.encode())]
        assert got == want
    got = w.process_documents("fast AND NOT best")              # operator words stay operators
    assert got == [{"document": {"name": o.doc_key(d).decode()}, "score": s}
                   for d, s in o.search(b"fast AND NOT best")] and got
    assert w.process_documents("fast AND") == []                # ParseException: Worker.java:182-185
    out = Leader([w]).start("fast food")
    assert list(out) == sorted(out)                              # TreeMap order
    assert list(out) == ["file.txt", "file3.txt", "file5.txt", "file6.txt", "file7.txt", "file8.txt"]
    assert w.get_index_size() > 0
    w.close()


def test_worker_latin1_file_goes_through_extractor(tmp_path):
    """A windows-1252 file (not UTF-8): Worker.java:199-211 hands it to Tika;
    the mirror's extractor decodes it and the index sees the UTF-8 text."""
    from tfidf_amd.reference_api import Worker
    docs = tmp_path / "documents"
    docs.mkdir()
    (docs / "a.txt").write_bytes(b"caf\xe9 cr\xe8me br\xfbl\xe9e")
    (docs / "b.txt").write_bytes("café noir".encode())
    w = Worker(str(docs), str(docs / ".luceneIndex"))
    w.init()
    assert [r["document"]["name"] for r in w.process_documents("café")] in (["a.txt", "b.txt"], ["b.txt", "a.txt"])
    assert [r["document"]["name"] for r in w.process_documents("crème")] == ["a.txt"]
    w.close()


# ---------------------------------------------------------------------------
# synthetic Zipf corpora

@pytest.fixture(scope="module")
def zipf():
    texts = synth.corpus(3000, V=20000, len_min=30, len_max=220)
    g, o = build_pair(texts)
    yield g, o, texts
    g.close()
    o.close()


def test_zipf_stats(zipf):
    g, o, _ = zipf
    s = g.stats()
    assert s["doc_count"] == o.doc_count
    assert s["sum_ttf"] == o.sum_ttf
    assert s["num_terms"] == o.num_terms
    assert s["long_docs"] == 0


def test_zipf_tf_rows(zipf):
    g, o, texts = zipf
    for d in list(range(0, 3000, 97)) + [2999]:
        assert g.doc_terms(d) == o.doc_terms(d)
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))


def test_zipf_df(zipf):
    g, o, _ = zipf
    vocab = o.vocab()
    rng = random.Random(3)
    for t in rng.sample(sorted(vocab), 400):
        assert g.df(t)[0] == vocab[t]


def test_zipf_queries_all_hits(zipf):
    g, o, _ = zipf
    for q in synth.queries(25, lo=1, hi=3000) + [b"aaaa", b"aaaa aaab aaac aaad"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))


def test_zipf_queries_topk_and_batch(zipf):
    g, o, _ = zipf
    qs = synth.queries(40, lo=1, hi=5000) + [b"aaaa aaab", b"zzzzz"]
    for k in (10, 100):
        docs, scores, counts = g.search_batch(qs, k)
        for i, q in enumerate(qs):
            want = o.search(q, k)
            got = list(zip(docs[i, :counts[i]].tolist(), scores[i, :counts[i]].tolist()))
            assert_hits_equal(got, want)
            assert_hits_equal(g.search(q, k), want)


def test_zipf_ties_many_equal_scores():
    # one short term repeated identically in many docs -> huge tie groups
    texts = [b"alpha beta" if i % 3 else b"alpha gamma delta" for i in range(20000)]
    g, o = build_pair(texts)
    for k in (0, 7, 1000):
        assert_hits_equal(g.search(b"alpha", k), o.search(b"alpha", k))
    g.close()
    o.close()


# ---------------------------------------------------------------------------
# tokenizer edge cases, long documents, updates, errors

ALPHABET = "abcXYZ019_:.',; -\n\t"


def random_text(rng, n):
    return "".join(rng.choice(ALPHABET) for _ in range(n)).encode()


def test_punctuation_corpus_parity():
    rng = random.Random(7)
    texts = [random_text(rng, rng.randint(0, 3000)) for _ in range(400)]
    texts += [b"", b"   ", b"___", b"...", b"a.b.c", b"3,14;15", b"don't", b"x" * 17, b"w" * 18, b"y" * 19, b"z" * 255]
    g, o = build_pair(texts)
    s = g.stats()
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"]) == (o.doc_count, o.sum_ttf, o.num_terms)
    for d in range(len(texts)):
        assert g.doc_terms(d) == o.doc_terms(d), d
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))
    for q in [b"a", b"b.c x", b"3,14", b"abc xyz", b"_", b"y" * 19]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()


def test_long_documents_path():
    rng = random.Random(11)
    cdf = synth.zipf_cdf(50000)
    texts = synth.corpus(200, V=50000, len_min=10, len_max=400)
    # long docs: > 4 KB and/or > 1024 tokens, up to ~120k tokens
    for n in (700, 1500, 5000, 40000, 120000):
        ranks = synth.doc_ranks(99, n, n, n, cdf)
        texts.insert(rng.randrange(len(texts)), b" ".join(synth.word(int(r)) for r in ranks))
    texts.insert(5, b"ab " * 2000)                  # 6 KB, 2000 tokens of one term
    texts.insert(9, random_text(rng, 20000))        # punctuation-heavy long doc
    g, o = build_pair(texts, cap_log2=18)
    s = g.stats()
    assert s["long_docs"] >= 6       # 700-token doc (< 4 KB) stays on the LDS path
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in range(len(texts)):
        if len(texts[d]) > 4096 or d % 17 == 0:
            assert g.doc_terms(d) == o.doc_terms(d), d
            assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))
    for q in synth.queries(15, lo=1, hi=2000) + [b"ab", b"a b c"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
        assert_hits_equal(g.search(q, 10), o.search(q, 10))
    g.close()
    o.close()


def test_update_document_replaces_by_key():
    texts = [b"fast food", b"cat meowing", b"night at night", b"fast cat"]
    keys = [b"a.txt", b"b.txt", b"a.txt", b"c.txt"]
    g, o = build_pair(texts, keys)
    assert g.stats()["num_docs"] == o.num_docs == 3
    assert [g.doc_key(d) for d in range(3)] == [o.doc_key(d) for d in range(3)] == [b"b.txt", b"a.txt", b"c.txt"]
    for q in [b"fast", b"night", b"cat"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()


def test_incremental_add_then_recommit():
    a = synth.corpus(500, V=3000, len_min=20, len_max=80)
    b = synth.corpus(300, V=3000, len_min=20, len_max=80, doc_base=500)
    g = ShardIndex()
    g.add_documents(a)
    g.commit()
    g.add_documents(b)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(a + b):
        o.add_doc(str(i).encode(), t)
    o.commit()
    for q in synth.queries(10, lo=1, hi=500):
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()


def test_host_loader_pinned_staging_and_clear():
    """Host corpus of > 2 staging buffers (32 MiB each) through the pinned
    loader = the same corpus added device-to-device; clear() empties the index
    and a re-add reproduces it."""
    dc = synth.DeviceCorpus(40000, V=50000, len_min=300, len_max=500)
    text, offs = dc.to_host()
    assert len(text) > 70 << 20
    a = ShardIndex()
    a.add_documents_buffer(text, offs)
    a.commit()
    b = ShardIndex()
    b.add_documents_device(dc.d_text, dc.d_offsets, dc.n_docs, dc.total_bytes)
    b.commit()
    sa = index_stats(a)
    assert sa == index_stats(b)
    qs = synth.queries(10)
    want = [b.search(q, 10) for q in qs]
    assert [a.search(q, 10) for q in qs] == want
    a.clear()
    assert a.stats()["num_docs"] == 0
    a.add_documents_buffer(text, offs)
    a.commit()
    assert index_stats(a) == sa
    assert [a.search(q, 10) for q in qs] == want
    # spot-check a few documents against the oracle
    o = O.OracleIndex()
    for d in (0, 17, 39999):
        o.add_doc(str(d).encode(), text[int(offs[d]):int(offs[d + 1])].tobytes())
    o.commit()
    for i, d in enumerate((0, 17, 39999)):
        assert a.doc_terms(d) == o.doc_terms(i)
    for x in (a, b, o):
        x.close()
    dc.free()


def test_malformed_utf8_document_indexed_empty():
    """A document that is not valid UTF-8 (Files.readString throws,
    Worker.java:199-211) is indexed with an empty field and listed — it does
    not fail the commit; the other documents are unaffected."""
    texts = [b"fine text", "caf\u00e9 au lait".encode(), b"caf\xe9 fine", b"ok \xff\xfe text", b"text again"]
    g, o = build_pair(texts, keys=[b"%d" % i for i in range(5)])
    assert g.malformed_docs() == o.malformed_docs() == [2, 3]
    s = g.stats()
    assert s["malformed_docs"] == 2 and s["num_docs"] == 5
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"]) == (o.doc_count, o.sum_ttf, o.num_terms) == (3, 7, 6)
    for d in range(5):
        assert g.doc_terms(d) == o.doc_terms(d)
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))
    for q in (b"fine", b"text", b"caf\xc3\xa9"):
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    # replace-by-key with the extracted text, then commit again
    g.add_documents([b"caf\xc3\xa9 fine"], [b"2"])
    g.commit()
    m = g.malformed_docs()                    # updateDocument: doc "3" is now id 2, "2" moved to the end
    assert [g.doc_key(d) for d in m] == [b"3"] and g.stats()["malformed_docs"] == 1
    assert g.doc_key(4) == b"2" and g.doc_len(4)[0] == 2
    g.close()
    o.close()


def test_empty_index_and_empty_docs():
    g = ShardIndex()
    g.add_documents([b"", b"  ..  ", b""])
    g.commit()
    s = g.stats()
    assert s["doc_count"] == 0 and s["num_terms"] == 0 and s["num_docs"] == 3
    assert g.search(b"anything", 0) == []
    g.close()


# ---------------------------------------------------------------------------
# GLOBAL statistics across shards (device vocabulary canonicalisation)

def test_global_stats_two_shards_equal_single_index():
    import torch
    texts = synth.corpus(4000, V=8000, len_min=20, len_max=120)
    halves = [texts[:1700], texts[1700:]]
    shards = []
    for h in halves:
        s = ShardIndex()
        s.add_documents(h)
        s.commit()
        shards.append(s)
    dev = torch.device("cuda:0")
    keys = []
    for s in shards:
        n = s.vocab_size()
        k = torch.zeros((n, 2), dtype=torch.int64, device=dev)
        df = torch.zeros(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        s.vocab_export_device(k.data_ptr(), df.data_ptr(), n)
        keys.append(k)
    all_keys = torch.cat(keys).contiguous()
    torch.cuda.synchronize()                      # the shards run on their own streams
    dfcs = []
    for s in shards:
        dfc = torch.zeros(all_keys.shape[0], dtype=torch.int32, device=dev)
        n = s.vocab_canonicalize_device(all_keys.data_ptr(), all_keys.shape[0], dfc.data_ptr(), all_keys.shape[0])
        dfcs.append(dfc[:n])
    assert dfcs[0].shape == dfcs[1].shape
    total = (dfcs[0] + dfcs[1]).contiguous()
    torch.cuda.synchronize()
    st = [s.stats() for s in shards]
    dc = sum(x["doc_count"] for x in st)
    ttf = sum(x["sum_ttf"] for x in st)
    for s in shards:
        s.set_global_stats_device(total.data_ptr(), total.shape[0], dc, ttf)
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    for q in synth.queries(20, lo=1, hi=2000):
        want = o.search(q, 0)
        got = []
        for base, s in zip((0, 1700), shards):
            got += [(d + base, sc) for d, sc in s.search(q, 0)]
        got.sort(key=lambda x: (-x[1], x[0]))
        assert_hits_equal(got, want)
    for s in shards:
        s.close()
    o.close()


def test_global_stats_term_ownership_three_shards():
    """The ownership exchange (vocab_partition -> all-to-all -> owner reduce ->
    all-to-all back -> import), with the all-to-alls done by hand between three
    shards on one GPU, equals the single index."""
    import torch
    texts = synth.corpus(5000, V=8000, len_min=20, len_max=120)
    cuts = [0, 1200, 3100, 5000]
    G = 3
    dev = torch.device("cuda:0")
    shards, recs, counts = [], [], []
    for r in range(G):
        s = ShardIndex()
        s.add_documents(texts[cuts[r]:cuts[r + 1]])
        s.commit()
        n = s.vocab_size()
        rec = torch.zeros((n, 3), dtype=torch.int64, device=dev)
        cnt = torch.zeros(G, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        n2 = s.vocab_partition_device(G, rec.data_ptr(), n, cnt.data_ptr())
        s.set_stream(None)                            # (asynchronous: finish the index's stream)
        c = cnt.cpu()
        assert n2 == n and int(c.sum()) == n
        shards.append(s)
        recs.append(rec)
        counts.append([int(x) for x in c])
    starts = [[sum(counts[r][:o]) for o in range(G)] for r in range(G)]
    answers = [[None] * G for _ in range(G)]          # answers[sender][owner]
    n_unique = 0
    for o in range(G):                                # owner o receives from every rank, in rank order
        parts = [recs[r][starts[r][o]:starts[r][o] + counts[r][o]] for r in range(G)]
        recv = torch.cat(parts).contiguous()
        out = torch.zeros(max(recv.shape[0], 1), dtype=torch.int32, device=dev)
        nu = torch.zeros(1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        shards[o].vocab_reduce_device(recv.data_ptr(), recv.shape[0], out.data_ptr(), nu.data_ptr())
        shards[o].set_stream(None)
        n_unique += int(nu.item())
        at = 0
        for r in range(G):
            answers[r][o] = out[at:at + counts[r][o]]
            at += counts[r][o]
    st = [s.stats() for s in shards]
    dc, ttf = sum(x["doc_count"] for x in st), sum(x["sum_ttf"] for x in st)
    for r in range(G):
        back = torch.cat(answers[r]).contiguous()
        torch.cuda.synchronize()
        shards[r].set_global_df_device(back.data_ptr(), back.shape[0], dc, ttf)
        shards[r].set_stream(None)
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    assert n_unique == o.num_terms
    vocab = o.vocab()
    for t in list(vocab)[:200]:
        for s in shards:
            loc, eff = s.df(t)
            assert eff == vocab[t] or loc == 0
    for q in synth.queries(20, lo=1, hi=2000):
        want = o.search(q, 0)
        got = []
        for base, s in zip(cuts, shards):
            got += [(d + base, sc) for d, sc in s.search(q, 0)]
        got.sort(key=lambda x: (-x[1], x[0]))
        assert_hits_equal(got, want)
    for s in shards:
        s.close()
    o.close()


# ---------------------------------------------------------------------------
# persistence (tfidf_save / tfidf_load; the reference reopens its FSDirectory index)

def test_save_load_roundtrip(tmp_path):
    texts = synth.corpus(3000, V=20000, len_min=20, len_max=150)
    keys = [b"d%d.txt" % (i % 2600) for i in range(3000)]         # 400 replaced keys
    g = ShardIndex()
    g.add_documents(texts, keys)
    g.commit()
    path = str(tmp_path / "ix.tfidf")
    g.save(path)
    h = ShardIndex()
    h.load(path)
    h.commit()
    assert index_stats(h) == index_stats(g)
    n = g.stats()["num_docs"]
    assert [h.doc_key(d) for d in range(0, n, 37)] == [g.doc_key(d) for d in range(0, n, 37)]
    for q in synth.queries(15, lo=1, hi=3000):
        assert h.search(q, 0) == g.search(q, 0)
    # appending after a reopen replaces by key, like the reference's CREATE_OR_APPEND writer
    more = synth.corpus(200, V=20000, len_min=20, len_max=150, doc_base=5000)
    mkeys = [b"d%d.txt" % i for i in range(100)] + [b"new%d.txt" % i for i in range(100)]
    h.add_documents(more, mkeys)
    h.commit()
    o = O.OracleIndex()
    for t, k in zip(texts + more, keys + mkeys):
        o.add_doc(k, t)
    o.commit()
    assert h.stats()["num_docs"] == o.num_docs
    for q in synth.queries(15, lo=1, hi=3000):
        assert_hits_equal(h.search(q, 0), o.search(q, 0))
    # corrupt / foreign files are refused
    bad = tmp_path / "bad.tfidf"
    bad.write_bytes(b"not an index")
    e = ShardIndex()
    with pytest.raises(Exception):
        e.load(str(bad))
    for x in (g, h, e, o):
        x.close()


def test_worker_restart_reopens_index(tmp_path, lucene_fixture):
    from tfidf_amd.reference_api import Worker
    docs = tmp_path / "documents"
    docs.mkdir()
    for d in lucene_fixture["docs"]:
        (docs / d["name"]).write_bytes(d["text"].encode())
    idx = str(docs / ".luceneIndex")
    w = Worker(str(docs), idx)
    w.init()
    before = w.process_documents("fast food")
    assert w.upload("extra.txt", b"fast food fast food truck")[0] == 200
    after = w.process_documents("fast food")
    w.close()
    w2 = Worker(str(docs), idx)                                   # restart: reopen + re-walk
    w2.init()
    assert w2.process_documents("fast food") == after != before
    names = [r["document"]["name"] for r in w2.process_documents("truck")]
    assert names == ["extra.txt"]
    w2.close()
