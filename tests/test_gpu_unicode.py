"""GPU parity of the full-Unicode tokenizer path.

Documents with a non-ASCII byte or a token of more than 255 chars leave the
ASCII wave path (and packed windows) for k_tokenize_long's general phase,
which rescans them with the device DFA of unicode_scan.h, thread slices cut
after ASCII class-OTHER bytes.  Checked against the CPU oracle
(oracle/tfidf_oracle.c: local join rules), itself pinned to a transcription of
the JFlex grammar (test_unicode_tokenizer.py).  Non-ASCII results are "parity
unpinned" against Lucene itself (no JDK here).  Bar: TF / DF / lengths / norms
/ hit ids bit-exact, scores as float32 bit patterns.
"""
import random

import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

from test_gpu_parity import assert_hits_equal
from test_unicode_tokenizer import ALPHA

pytestmark = pytest.mark.gpu

WORDS = ["café", "Café", "naïve", "it’s", "don't", "élan", "ÉCOLE", "straße", "İstanbul", "ΣΟΦΙΑ", "σοφία",
         "москва", "Москва", "中文", "分词器", "ひらがな", "カタカナ", "ภาษาไทย", "שָׁלוֹם", "א\"ב", "١٢٫٣", "１２３",
         "😀", "👍🏽", "👨‍👩‍👧", "🇺🇸", "été", "abc", "xyz", "42", "u.s.a", "q_1"]


def uni_doc(rng, n):
    parts = []
    for _ in range(n):
        r = rng.random()
        if r < 0.6:
            parts.append(rng.choice(WORDS))
        elif r < 0.8:
            parts.append("".join(rng.choice(ALPHA) for _ in range(rng.randint(1, 8))))
        else:
            parts.append(synth.word(rng.randint(1, 3000)).decode())
        parts.append(rng.choice([" ", " ", " ", "\n", ", ", " — ", "　", "\t"]))
    return "".join(parts).encode()


def build_pair(texts, cap_log2=18):
    g = ShardIndex(vocab_capacity_log2=cap_log2)
    g.add_documents(texts)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    return g, o


def check(g, o, texts, every=1):
    s = g.stats()
    assert (s["doc_count"], s["sum_ttf"], s["num_terms"], s["nnz"]) == \
        (o.doc_count, o.sum_ttf, o.num_terms, sum(o.vocab().values()))
    for d in range(0, len(texts), every):
        assert g.doc_terms(d) == o.doc_terms(d), (d, texts[d][:200])
        assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d)), d


QUERIES = ["café", "CAFÉ naïve", "it’s", "中文 分词器", "ภาษาไทย", "😀 🇺🇸", "σοφία ΣΟΦΙΑ", "москва abc",
           "straße　42", "été", "א\"ב", "１２３ u.s.a"]


def test_mixed_corpus_short_and_long_docs():
    rng = random.Random(5)
    texts = [uni_doc(rng, rng.randint(0, 300)) for _ in range(600)]
    texts += synth.corpus(400, V=3000, len_min=20, len_max=300)          # ASCII docs stay on the wave path
    texts += [uni_doc(rng, n) for n in (2000, 9000, 30000)]             # long Unicode docs (> 4 KB)
    rng.shuffle(texts)
    texts += [b"", "　".encode(), "﻿".encode(), "ั".encode(), "_ั".encode()]
    g, o = build_pair(texts)
    st = g.stats()
    assert st["unicode_docs"] >= 550 and st["long_docs"] < 100    # short Unicode docs: the Unicode wave path
    check(g, o, texts)
    for q in QUERIES:
        qb = q.encode()
        assert_hits_equal(g.search(qb, 0), o.search(qb, 0))
        assert_hits_equal(g.search(qb, 10), o.search(qb, 10))
    docs, scores, counts = g.search_batch([q.encode() for q in QUERIES], 10)
    for i, q in enumerate(QUERIES):
        hits = list(zip(docs[i, :counts[i]].tolist(), scores[i, :counts[i]].tolist()))
        assert_hits_equal(hits, o.search(q.encode(), 10))
    g.close()
    o.close()


@pytest.mark.parametrize("pack", [4, 16])
def test_packed_windows_defer_unicode_docs(monkeypatch, pack):
    monkeypatch.setenv("TFIDF_PACK_DOCS", str(pack))
    rng = random.Random(pack)
    texts = []
    for i in range(1500):
        texts.append(uni_doc(rng, rng.randint(1, 12)) if i % 7 == 3 else
                     b" ".join(synth.word(rng.randint(1, 500)) for _ in range(rng.randint(1, 12))))
    g, o = build_pair(texts)
    assert g.stats()["pack_docs"] == pack
    check(g, o, texts)
    g.close()
    o.close()


def test_tokens_longer_than_255_chars_are_cut():
    rng = random.Random(9)
    texts = [b"x" * 256, b"ab " + b"y" * 600 + b" cd", ("é" * 300).encode(), (b"q" * 254 + "\U00010400".encode() * 3),
             b"a.b" * 120, b"_" * 300 + b"z", b"k" * 255, b"fine text only"]
    texts += [b" ".join([b"w" * rng.randint(200, 700)] * 3) for _ in range(20)]
    texts += synth.corpus(300, V=500, len_min=5, len_max=50)
    g, o = build_pair(texts)
    check(g, o, texts)
    for q in [b"x" * 255, b"y" * 255, "é" * 255, b"k" * 255, b"fine"]:
        qb = q if isinstance(q, bytes) else q.encode()
        assert_hits_equal(g.search(qb, 0), o.search(qb, 0))
    g.close()
    o.close()


def test_whitespace_free_unicode_document():
    # no ASCII split byte at all: the first thread slice scans the whole document
    rng = random.Random(2)
    t = "".join(rng.choice("中文字ひらがなカタカナภาษา") for _ in range(20000)).encode()
    texts = [t, "東京タワー".encode() * 500, b"plain words here"]
    g, o = build_pair(texts)
    check(g, o, texts)
    g.close()
    o.close()


def test_book_corpus_long_unicode_docs():
    # SURVEY cfg 1 shape (a few hundred books; here 12 of ~240 KB): every
    # document takes the long path's general phase; AUTO builds term-major
    # (too few (block, range) tiles for the block-major passes).
    rng = random.Random(12)
    texts = [uni_doc(rng, rng.randint(20000, 40000)) for _ in range(10)]
    texts += [b" ".join(synth.word(rng.randint(1, 20000)) for _ in range(30000))] * 2
    g, o = build_pair(texts)
    st = g.stats()
    assert st["long_docs"] == len(texts) and st["term_major"] == 1
    check(g, o, texts)
    for q in QUERIES + [synth.word(5).decode() + " " + synth.word(77).decode()]:
        qb = q.encode()
        assert_hits_equal(g.search(qb, 0), o.search(qb, 0))
        assert_hits_equal(g.search(qb, 3), o.search(qb, 3))
    g.close()
    o.close()


def test_book_unicode_chunks():
    """Books (cfg 1 shape) whose text is mostly ASCII with a non-ASCII word
    every few hundred words (curly apostrophes, accents, a CJK pair, an emoji):
    the units holding non-ASCII text take the Unicode chunk kernel
    (k_tokenize_uchunk) and the book stays on the chunk path instead of going
    to k_tokenize_long whole; one book with an unspaced CJK run longer than a
    unit's leading margin falls back to the long path for that book.  All =
    the oracle."""
    rng = random.Random(21)
    sprinkle = ["it’s", "don’t", "café", "naïve", "Élan", "straße", "中文", "😀", "ΣΟΦΙΑ", "ﬁne"]
    texts = []
    for i in range(9):
        words = [synth.word(rng.randint(1, 20000)).decode() for _ in range(rng.randint(20000, 40000))]
        for j in range(rng.randint(0, 50), len(words), rng.randint(150, 450)):
            words[j] = rng.choice(sprinkle)
        texts.append(" ".join(words).encode())
    cjk = " ".join(synth.word(rng.randint(1, 5000)).decode() for _ in range(6000))
    texts.append((cjk + " " + "中文分词器" * 300 + " " + cjk).encode())      # 4.5 KB without a split byte
    g, o = build_pair(texts)
    st = g.stats()
    assert st["long_docs"] == len(texts)
    assert st["long_chunked"] == len(texts) - 1                         # only the CJK book goes to the long path
    check(g, o, texts)
    for q in ["café it’s", "naïve straße", "中文 " + synth.word(7).decode(), "ﬁne 😀", synth.word(99).decode()]:
        qb = q.encode()
        assert_hits_equal(g.search(qb, 0), o.search(qb, 0))
        assert_hits_equal(g.search(qb, 5), o.search(qb, 5))
    g.close()
    o.close()


def prose_book(rng, n_words):
    """Book-like prose: sentence capitals, ALL-CAPS names, curly and ASCII
    quotes / apostrophes, em dashes, numbers with separators ("1,000", "3.14"),
    letter-digit mixes, hyphens, ellipses, snake_case, accented words in mixed
    case — the characters real books put between and inside ASCII words."""
    accented = ["Émile", "ÉCOLE", "café", "Café", "naïve", "façade", "Zoë", "señor", "Über", "übermäßig", "ﬁnal"]
    out, cap = [], True
    for _ in range(n_words):
        r = rng.random()
        if r < 0.04:
            w = rng.choice(accented)
        elif r < 0.07:
            w = rng.choice(["1,000", "3.14", "2024", "12:30", "A4", "x86_64", "v2.0", "1,234,567.89", "4th"])
        elif r < 0.10:
            w = rng.choice(["it’s", "don’t", "can't", "O’Neil", "rock’n’roll", "l’été", "we'd"])
        elif r < 0.12:
            w = synth.word(rng.randint(1, 3000)).decode() + "-" + synth.word(rng.randint(1, 3000)).decode()
        elif r < 0.13:
            w = synth.word(rng.randint(1, 800)).decode().upper()
        elif r < 0.135:
            w = "snake_" + synth.word(rng.randint(1, 500)).decode()
        else:
            w = synth.word(rng.randint(1, 20000)).decode()
        if cap:
            w = w[:1].upper() + w[1:]
            cap = False
        q = rng.random()
        if q < 0.03:
            w = "“" + w + "”"
        elif q < 0.05:
            w = "\"" + w + "\""
        elif q < 0.06:
            w = "‘" + w + "’"
        out.append(w)
        p = rng.random()
        if p < 0.06:
            out.append(rng.choice([". ", "! ", "? ", "… ", "... "]))
            cap = True
        elif p < 0.10:
            out.append(rng.choice([", ", "; ", ": ", " — ", "—", " – ", " (", ") "]))
        elif p < 0.11:
            out.append("\n\n")
            cap = True
        else:
            out.append(" ")
    return "".join(out).encode()


def test_book_prose_unicode_chunks():
    """Books of realistic prose (curly quotes, em dashes, contractions with
    U+2019, accented capitals, numbers with separators) on the chunk path: the
    Unicode chunk kernel's ASCII shortcuts (runs of letters / digits skipped in
    the DFA's A / N states, keys of <= 8 ASCII bytes built directly) meet every
    join rule (WB6/7 MidLetter, WB11/12 MidNum, MidNumLet, Single_Quote,
    ExtendNumLet) next to non-ASCII characters.  All = the oracle."""
    rng = random.Random(33)
    texts = [prose_book(rng, rng.randint(12000, 22000)) for _ in range(8)]
    texts += [prose_book(rng, rng.randint(50, 400)) for _ in range(200)]        # short documents: the Unicode wave
    g, o = build_pair(texts)
    st = g.stats()
    assert st["long_docs"] >= 8 and st["long_chunked"] >= 8
    check(g, o, texts)
    for q in ["café Émile", "it’s don’t", "1,000 3.14", "ÉCOLE école", "rock’n’roll", "snake_" + synth.word(3).decode(),
              "x86_64 v2.0", synth.word(12).decode() + " " + synth.word(400).decode(), "o’neil über"]:
        qb = q.encode()
        assert_hits_equal(g.search(qb, 0), o.search(qb, 0))
        assert_hits_equal(g.search(qb, 7), o.search(qb, 7))
    g.close()
    o.close()
