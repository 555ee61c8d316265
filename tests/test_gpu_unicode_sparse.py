"""The Unicode wave path's sparse form (round 5, kernels_unicode.hip
uw_sparse_tokens): in a document with a few non-ASCII chars, the ASCII words
take the wave tokenizer's SWAR rules and only the "islands" — the pieces
between ASCII class-OTHER bytes that hold a byte >= 0x80 — take the
longest-match scanner.  Checked against the CPU oracle (oracle/tfidf_oracle.c,
pinned to the JFlex grammar transcription in test_unicode_tokenizer.py) with
the sparse form on and forced off (TFIDF_UW_FULL=1: the whole-document scan),
on documents built to put islands next to every joiner, at document and
64-byte lane edges, and past the sparse form's limits (it must fall back).
Bar: TF / DF / lengths / norms / hits bit-exact.
"""
import random

import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

from test_gpu_parity import assert_hits_equal

pytestmark = pytest.mark.gpu

EDGE = ["l'été", "café's", "end.é", "é.end", "a.é.b", "3,é", "é3,5", "__é__", "_é", "é_", "naïve_user",
        "über.cool", "x’s", "don’t", "école", "́abc", "abc­def", "a b", "中文abc", "abc中文",
        "😀abc", "abc😀", "İstanbul", "ΣΟΦΙΑ", "ﬁne", "a:é", "é:a", "1.é", "é'1", "_‍_", "x‍y",
        "q\"é", "é\"q", "ab;é;cd", "ÀB.CD", "a_1_é"]
SEPS = [" ", " ", "\n", ", ", ". ", " - ", "(", ") ", "\t", "; ", ": ", "'"]


def sparse_doc(rng, n_words, n_uni):
    words = [synth.word(rng.randint(1, 4000)).decode() for _ in range(n_words)]
    for _ in range(n_uni):
        words.insert(rng.randint(0, len(words)), rng.choice(EDGE))
    out = []
    for w in words:
        out.append(w)
        out.append(rng.choice(SEPS))
    return "".join(out).encode()


def edge_docs():
    docs = []
    for w in EDGE:
        docs += [w, w + " tail", "head " + w, "head " + w + " tail", w + w, w + "." + w]
    # islands across the 64-byte lane edges and at the window's end
    for pad in range(56, 70):
        docs.append("a" * pad + " é " + "b" * 10)
        docs.append("x " * (pad // 2) + "naïve")
    docs.append(("word " * 800)[:4000] + " café")                  # near the 4 KB window
    docs.append("é " + "z" * 300 + " abc")                          # ASCII token > 255 chars: full scan
    docs.append(" ".join(["é%d" % i for i in range(100)]))          # > 64 islands: full scan
    docs.append("x" * 600 + "é")                                    # piece > 512 bytes: full scan
    docs.append("bad \xff byte é")                                  # not UTF-8 (bytes below)
    return [d.encode("utf-8", "surrogateescape") if isinstance(d, str) else d for d in docs]


def build_pair(texts):
    g = ShardIndex()
    g.add_documents(texts)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    return g, o


def check(g, o, texts):
    s = g.stats()
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    assert g.malformed_docs() == o.malformed_docs()
    for d in range(len(texts)):
        assert g.doc_terms(d) == o.doc_terms(d), (d, texts[d][:200])
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d)), d


@pytest.mark.parametrize("full", [False, True])
def test_sparse_unicode_docs_equal_oracle(monkeypatch, full):
    if full:
        monkeypatch.setenv("TFIDF_UW_FULL", "1")
    rng = random.Random(31)
    texts = edge_docs()
    texts[-1] = b"bad \xff byte \xc3\xa9"
    texts += [sparse_doc(rng, rng.randint(20, 500), rng.randint(1, 6)) for _ in range(800)]
    texts += synth.corpus(200, V=4000, len_min=50, len_max=400)       # pure ASCII: the wave path
    rng.shuffle(texts)
    g, o = build_pair(texts)
    assert g.stats()["unicode_docs"] >= 800
    check(g, o, texts)
    for q in ["été", "café", "naïve_user", "über cool", "don’t", "école", "中文 abc", "ﬁne", "a_1_é", "istanbul",
              "σοφια", "x’s", synth.word(7).decode() + " é"]:
        qb = q.encode()
        for k in (0, 10):
            assert_hits_equal(g.search(qb, k), o.search(qb, k))
    g.close()
    o.close()
