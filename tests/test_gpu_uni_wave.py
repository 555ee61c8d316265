"""Non-ASCII documents by the wave rules (round 5, kernels_index.hip
k_tokenize_wave<UNI>): a document the ASCII pass flagged whose non-ASCII
chars are all well-formed ALetter code points that are their own lower case
(é ü ñ ß ø α я ...) is tokenized by the SWAR word rules with those bytes read
as letters; its tokens holding a non-ASCII byte take folded table keys and the
Unicode key builder.  Everything else (upper case, Han, Katakana, Hebrew,
combining marks, emoji, malformed bytes) stays with k_tokenize_uwave.

Checked against the CPU oracle (oracle/tfidf_oracle.c, the checker) with the
wave rules on and off (TFIDF_NO_UNIWAVE=1: every flagged document to the
Unicode wave path), on documents that put simple letters next to every
joiner, at the 64-byte lane edges (a char split across two lanes), in tokens
of <= 8 and > 8 bytes, mixed with ASCII case variants of the same term, and
next to documents the wave rules must decline.  Bar: TF / DF / lengths /
norms / hits bit-exact, and the declined documents counted apart.
"""
import random

import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

from test_gpu_parity import assert_hits_equal
from test_gpu_unicode_sparse import build_pair, check

pytestmark = pytest.mark.gpu

SIMPLE = ["é", "ü", "ñ", "ß", "ø", "å", "ł", "ş", "α", "ω", "я", "ж", "ə", "ŋ", "ǆ", "ﬁ"]
WORDS = ["café", "naïve", "über", "mañana", "straße", "smørrebrød", "kraków", "ελλάδα", "москва",
         "résumé", "déjà", "façade", "jalapeño", "crème", "brûlée", "coöperate", "zoë", "fiancée"]
JOIN = ["l'été", "café's", "end.é", "é.end", "a.é.b", "3,é", "é3,5", "__é__", "_é", "é_", "naïve_user",
        "über.cool", "a:é", "é:a", "1.é", "é'1", "ab;é;cd", "a_1_é", "Café", "CAFÉ".lower(), "NAÏVE".lower(),
        "CaFé", "x.y.ü", "ü,3", "a'b'é"]
DECLINE = ["中文", "カタカナ", "שלום", "é́", "😀", "İ", "­", "١٢٣", "a\u202fb", "©", "™", "x\u200dy", "‿"]
# Round 6, real prose: upper-case letters whose lower case has the same UTF-8
# length (lowered in the staged window), separators of class Other (curly
# double quotes, dashes, ellipsis, no-break space, guillemets: spaces), and
# non-ASCII mid chars (’ ‘ · ‧ ․ ＇: joined as ASCII ' . : are) — next to
# letters, digits, '_', ASCII joiners, each other, and at token edges.
PROSE = ["don’t", "it’s", "‘quoted’", "“quote”", "a—b", "x–y", "wait…", "non\u00a0breaking", "«guillemets»",
         "É", "Über", "ΣΟΦΙΑ", "École", "ÀÉÎÕÜ", "l’été", "3’4", "a’’b", "’tis", "rock’n’roll", "o’", "’",
         "a·b", "1·2", "x‧y", "a’1", "1’a", "a’.b", "a.’b", "_’a", "a’_", "Ça va", "QUÉBEC", "naïve—ok",
         "end.”", "“start", "a\u00a0’b", "‘a’", "9’", "’9", "A’B", "Ünïcödé’s", "x․y", "1․5", "x＇y", "a”b",
         "“É”", "—", "…", "a…b", "ΑΒΓ’δ", "Straße’s", "‘’", "a‘b", "1‘2", "a·1", "I’m", "O’NEIL", "L’ÉTÉ"]
SEPS = [" ", " ", "\n", ", ", ". ", " - ", "(", ") ", "\t", "; ", ": ", "'"]


def doc(rng, n_words, n_uni, pool):
    words = [synth.word(rng.randint(1, 3000)).decode() for _ in range(n_words)]
    for _ in range(n_uni):
        words.insert(rng.randint(0, len(words)), rng.choice(pool))
    out = []
    for w in words:
        out.append(w)
        out.append(rng.choice(SEPS))
    return "".join(out).encode()


def edge_docs():
    docs = []
    for w in WORDS + JOIN + SIMPLE:
        docs += [w, w + " tail", "head " + w, w + w, w + "." + w, w.upper().lower() + " " + w]
    # a 2-, 3- or 4-byte char across every lane edge and the window's end
    for ch in ["é", "я", "ǆ", "ə"]:
        for pad in range(58, 70):
            docs.append("a" * pad + ch + "b" * 12)
            docs.append("x " * (pad // 2) + "z" + ch + "z")
    docs.append(("word " * 800)[:4090] + " é")
    docs.append("é " + "z" * 300 + " abc")                         # > 255 chars: the long path cuts it
    docs.append("é" * 200)                                           # 400 bytes, 200 units: one token
    docs.append(" ".join("é%d" % i for i in range(300)))             # many distinct non-ASCII terms
    return [d.encode() for d in docs]


@pytest.mark.parametrize("uniwave", [True, False])
def test_simple_non_ascii_docs_equal_oracle(monkeypatch, uniwave):
    if not uniwave:
        monkeypatch.setenv("TFIDF_NO_UNIWAVE", "1")
    rng = random.Random(71)
    texts = edge_docs()
    simple = [doc(rng, rng.randint(20, 500), rng.randint(1, 8), WORDS + JOIN + SIMPLE) for _ in range(900)]
    declined = [doc(rng, rng.randint(20, 300), 1, DECLINE) for _ in range(150)]
    texts += simple + declined
    texts += synth.corpus(200, V=3000, len_min=50, len_max=400)     # pure ASCII
    rng.shuffle(texts)
    g, o = build_pair(texts)
    st = g.stats()
    assert st["unicode_docs"] >= 900 + 150
    if uniwave:
        assert st["unicode_wave_docs"] >= 900                         # the simple ones went the wave way
        assert st["unicode_docs"] - st["unicode_wave_docs"] >= 150    # the declined ones did not
    else:
        assert st["unicode_wave_docs"] == 0
    check(g, o, texts)
    for q in ["café", "naïve", "über cool", "straße", "ελλάδα", "москва", "résumé déjà", "l'été", "a_1_é",
              "CAFÉ", "Über", "中文", synth.word(5).decode() + " é", "é"]:
        qb = q.encode()
        for k in (0, 10):
            assert_hits_equal(g.search(qb, k), o.search(qb, k))
    g.close()
    o.close()


def test_same_term_across_paths():
    """A term spelled in a document the wave rules take and in one they decline
    (an upper-case É elsewhere in it) is one dictionary term: df 2, one
    posting list."""
    texts = [b"caf\xc3\xa9 au lait", "CAFÉ noir 中".encode(), "Café crème".encode(), "café".encode() * 3]
    g, o = build_pair(texts)
    st = g.stats()
    assert st["unicode_wave_docs"] >= 2 and st["unicode_docs"] - st["unicode_wave_docs"] >= 1
    check(g, o, texts)
    assert_hits_equal(g.search("café".encode(), 0), o.search("café".encode(), 0))
    g.close()
    o.close()


def test_cfg2_share_of_simple_docs_equal_oracle():
    """bench.py --unicode-frac's documents (one é word each) at a reduced size."""
    texts = synth.corpus(3000, V=5000, len_min=100, len_max=300)
    rng = random.Random(5)
    out = []
    for t in texts:
        if rng.random() < 0.5:
            w = t.split(b" ")
            i = rng.randrange(len(w))
            w[i] = w[i] + "é".encode()
            t = b" ".join(w)
        out.append(t)
    g, o = build_pair(out)
    st = g.stats()
    assert st["unicode_wave_docs"] == st["unicode_docs"] > 1000
    check(g, o, out)
    g.close()
    o.close()


@pytest.mark.parametrize("uniwave", [True, False])
def test_books_with_simple_non_ascii_words_equal_oracle(monkeypatch, uniwave):
    """Book-sized documents (the chunk path, 2 KB core units): units holding
    simple non-ASCII words go the wave way (k_tokenize_chunk<UNI>), units
    with other non-ASCII text to k_tokenize_uchunk, in one book."""
    if not uniwave:
        monkeypatch.setenv("TFIDF_NO_UNIWAVE", "1")
    rng = random.Random(13)
    texts = []
    for b in range(24):
        n_words = rng.randint(4000, 12000)
        pool = WORDS + JOIN + SIMPLE + (DECLINE if b % 4 == 0 else [])
        texts.append(doc(rng, n_words, n_words // 300, pool))
    texts += [doc(rng, rng.randint(20, 200), 1, WORDS) for _ in range(100)]
    g, o = build_pair(texts)
    check(g, o, texts)
    for q in ["café", "naïve", "straße", "москва", "l'été", "CAFÉ", "中文", synth.word(9).decode()]:
        qb = q.encode()
        for k in (0, 10):
            assert_hits_equal(g.search(qb, k), o.search(qb, k))
    g.close()
    o.close()


def prose_edge_docs():
    docs = []
    for w in PROSE:
        docs += [w, w + " tail", "head " + w, w + w, w + "." + w, "x" + w + "y", "1" + w + "2"]
    # each prose char across every lane edge and the window's end
    for ch in ["’", "—", "“", "\u00a0", "É", "·", "…", "Ω"]:
        for pad in range(58, 71):
            docs.append("a" * pad + ch + "b" * 12)
            docs.append("3" * pad + ch + "4" * 5)
            docs.append("x " * (pad // 2) + "z" + ch + "z")
    docs.append(("word " * 800)[:4088] + "’s")
    return [d.encode() for d in docs]


@pytest.mark.parametrize("uniwave", [True, False])
def test_prose_docs_equal_oracle(monkeypatch, uniwave):
    """Real prose (round 6): curly quotes and apostrophes, dashes, no-break
    spaces and capitalised accented letters take the wave rules too; declined
    characters still go to the Unicode wave path."""
    if not uniwave:
        monkeypatch.setenv("TFIDF_NO_UNIWAVE", "1")
    rng = random.Random(97)
    texts = prose_edge_docs()
    prose = [doc(rng, rng.randint(20, 500), rng.randint(1, 12), PROSE + WORDS + JOIN) for _ in range(900)]
    declined = [doc(rng, rng.randint(20, 300), 2, PROSE) + " 中文".encode() for _ in range(100)]
    texts += prose + declined
    texts += synth.corpus(200, V=3000, len_min=50, len_max=400)
    rng.shuffle(texts)
    g, o = build_pair(texts)
    st = g.stats()
    if uniwave:
        assert st["unicode_wave_docs"] >= 900
        assert st["unicode_docs"] - st["unicode_wave_docs"] >= 100
    else:
        assert st["unicode_wave_docs"] == 0
    check(g, o, texts)
    for q in ["don’t", "l’été", "québec", "École", "rock’n’roll", "a·b", "3’4", "“quote”", "Über", "ΣΟΦΙΑ",
              "o’neil", "wait", "naïve", "i’m"]:
        qb = q.encode()
        for k in (0, 10):
            assert_hits_equal(g.search(qb, k), o.search(qb, k))
    g.close()
    o.close()


@pytest.mark.parametrize("uniwave", [True, False])
def test_prose_books_equal_oracle(monkeypatch, uniwave):
    """Book-sized prose (the chunk units): no book goes to the long path when
    its non-ASCII text is prose."""
    if not uniwave:
        monkeypatch.setenv("TFIDF_NO_UNIWAVE", "1")
    rng = random.Random(31)
    texts = [doc(rng, rng.randint(4000, 12000), rng.randint(40, 120), PROSE + WORDS) for _ in range(16)]
    texts += [doc(rng, rng.randint(20, 200), 2, PROSE) for _ in range(100)]
    g, o = build_pair(texts)
    check(g, o, texts)
    if uniwave:
        st = g.stats()
        assert st["long_chunked"] == st["long_docs"] >= 16          # every book by its chunk units
    for q in ["don’t", "l’été", "québec", "rock’n’roll", synth.word(9).decode()]:
        qb = q.encode()
        for k in (0, 10):
            assert_hits_equal(g.search(qb, k), o.search(qb, k))
    g.close()
    o.close()


@pytest.mark.parametrize("unifirst", [True, False])
def test_uni_first_recommit_equals_oracle(monkeypatch, unifirst):
    """A re-commit after a commit whose documents were mostly non-ASCII runs
    UNI-first (round 6): every document starts flagged and the UNI wave pass
    takes the ASCII ones too (no ASCII pass); documents it declines (Han, too
    long for a wave window, malformed) still reach the Unicode wave and long
    paths.  Both commits, and the same re-commit without the mode
    (TFIDF_NO_UNIFIRST), equal the oracle; the non-ASCII count is unchanged."""
    if not unifirst:
        monkeypatch.setenv("TFIDF_NO_UNIFIRST", "1")
    rng = random.Random(113)
    texts = [doc(rng, rng.randint(20, 500), rng.randint(1, 12), PROSE + WORDS + JOIN) for _ in range(700)]
    texts += [doc(rng, rng.randint(20, 300), 2, PROSE) + " 中文".encode() for _ in range(60)]
    texts += synth.corpus(300, V=3000, len_min=50, len_max=400)                       # ASCII
    texts += [(" ".join(synth.word(rng.randint(1, 3000)).decode() for _ in range(2500))).encode()]   # > 4 KB
    texts += [b"bad \xff byte", ("word " * 820).encode(), prose_edge_docs()[7]]
    rng.shuffle(texts)
    g, o = build_pair(texts)
    st1 = g.stats()
    check(g, o, texts)
    g.commit()                                        # the same documents again: UNI-first unless disabled
    st2 = g.stats()
    check(g, o, texts)
    for k in ("unicode_docs", "unicode_wave_docs", "long_docs", "nnz", "num_terms"):
        if k in st1:
            assert st1[k] == st2[k], k
    for q in ["don’t", "québec", "École", "Über", "中文", synth.word(11).decode(), "word"]:
        qb = q.encode()
        for kk in (0, 10):
            assert_hits_equal(g.search(qb, kk), o.search(qb, kk))
    g.close()
    o.close()


def test_prose_chars_cut_by_chunk_windows_equal_oracle():
    """Round 6: a book unit's window (64 B before its 2 KB core, 320 B after)
    that cuts a multi-byte character in its margin blanks the cut bytes
    instead of declining the unit.  Books with a 2-, 3- or 4-byte character
    at every offset around each window edge (and around the core edges),
    inside words and between them: tokens equal the oracle's."""
    rng = random.Random(211)
    chars = ["’", "—", "é", "É", "…", " ", "·", "𝐀"]
    texts = []
    for b in range(12):
        n = 9000 + 500 * b
        buf = bytearray()
        while len(buf) < n:
            buf += synth.word(rng.randint(1, 3000)) + b" "
        buf = buf[:n]
        edges = []
        for k in range(1, n // 2048 + 1):
            edges += [2048 * k - 64, 2048 * k, 2048 * k + 2048 + 320, 2048 * k + 2048]
        ch = chars[b % len(chars)].encode()
        last = -10
        for e in sorted(set(edges)):
            p = e - rng.randint(0, len(ch)) - (b % 3)          # the char straddles (or touches) the edge
            if max(1, last + 1) <= p and p + len(ch) < len(buf) - 1:
                buf[p:p + len(ch)] = ch
                last = p + len(ch)
        t = bytes(buf)
        t.decode()                                             # still well-formed UTF-8
        texts.append(t)
    texts += [doc(rng, rng.randint(20, 200), 2, PROSE) for _ in range(50)]
    g, o = build_pair(texts)
    check(g, o, texts)
    st = g.stats()
    assert st["long_chunked"] == st["long_docs"] >= 12
    g.close()
    o.close()
