"""Full-Unicode StandardTokenizer (CPU): three formulations must agree.

1. a transcription of the JFlex grammar of Lucene 9.8.0 StandardTokenizerImpl
   (the WORD / SEA / IDEOGRAPHIC / HIRAGANA / EMOJI rules, each class X meaning
   X (Extend | Format | ZWJ)*) as a POSIX leftmost-LONGEST regex (the `regex`
   module), scanned like JFlex: longest rule match at the position, else skip
   one char;
2. the CPU oracle (oracle/tfidf_oracle.c: local join rules between units);
3. the engine (tfidf_analyze: the longest-match DFA of unicode_scan.h that the
   index build runs on the device).

Character classes for all three come from tools/gen_unicode_tables.py (ICU 70
properties of code points assigned in Unicode 9.0 = the grammar's
`%unicode 9.0`; JDK 17 lower-casing).  No Lucene runs here, so non-ASCII
tokenization is "parity unpinned" against the reference itself: what is
pinned is the grammar transcription (1) and, on ASCII, the golden fixture
(test_oracle_golden.py).
"""
import os
import random
import re

import pytest

from oracle import oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
regex = pytest.importorskip("regex")

CLASSES = ["OTHER", "ALETTER", "HEBREW", "NUMERIC", "KATAKANA", "EXTNUMLET", "MIDLETTER", "MIDNUMLET",
           "MIDNUM", "SQUOTE", "DQUOTE", "EXTEND", "EXTEND_SA", "ZWJ", "SA", "HAN", "HIRAGANA", "RI", "EMOJI"]


def _ranges():
    txt = open(os.path.join(REPO, "oracle", "unicode_props.h")).read()
    body = txt[txt.index("uc_ranges"):txt.index("UC_NRANGES")]
    out = {k: [] for k in CLASSES}
    for a, b, k in re.findall(r"\{0x([0-9A-F]+), 0x([0-9A-F]+), (\d+)\}", body):
        out[CLASSES[int(k)]].append((int(a, 16), int(b, 16)))
    return out


R = _ranges()


def cset(*names):
    parts = []
    for n in names:
        for a, b in R[n]:
            parts.append(regex.escape(chr(a)) if a == b else "%s-%s" % (regex.escape(chr(a)), regex.escape(chr(b))))
    return "[" + "".join(parts) + "]"


def grammar():
    X = "%s*" % cset("EXTEND", "EXTEND_SA", "ZWJ")
    ex = lambda *n: "(?:%s%s)" % (cset(*n), X)
    AHL, HL, NU, KA, ENL = ex("ALETTER", "HEBREW"), ex("HEBREW"), ex("NUMERIC"), ex("KATAKANA"), ex("EXTNUMLET")
    MIDL, MIDN = ex("MIDLETTER", "MIDNUMLET", "SQUOTE"), ex("MIDNUM", "MIDNUMLET", "SQUOTE")
    SQ, DQ = ex("SQUOTE"), ex("DQUOTE")
    core = ("(?:{KA}(?:{ENL}*{KA})*|(?:{HL}(?:{SQ}|{DQ}{HL})|{NU}(?:(?:{ENL}*|{MIDN}){NU})*"
            "|{AHL}(?:(?:{ENL}*|{MIDL}){AHL})*)+)").format(**locals())
    word = "{ENL}*{core}(?:{ENL}+{core})*{ENL}*".format(ENL=ENL, core=core)
    sea = "(?:%s%s)+" % (cset("SA", "EXTEND_SA"), X)
    ideo = ex("HAN")
    hira = ex("HIRAGANA")
    emo = "%s(?:%s*%s%s)*%s" % (cset("EMOJI"), cset("EXTEND", "EXTEND_SA", "ZWJ"), cset("ZWJ"), cset("EMOJI"), X)
    ri = "%s%s" % (ex("RI"), ex("RI"))
    return regex.compile("|".join("(?:%s)" % r for r in (word, sea, ideo, hira, emo, ri)), regex.POSIX)


G = grammar()


def jflex_tokens(s: str, max_len=255):
    """Scan like the generated JFlex scanner: longest match, else [^]."""
    out, i = [], 0
    while i < len(s):
        m = G.match(s, i)
        if not m or m.end() == i:
            i += 1
            continue
        tok, u16, k = [], 0, i
        while k < m.end() and u16 + (2 if ord(s[k]) > 0xFFFF else 1) <= max_len:
            u16 += 2 if ord(s[k]) > 0xFFFF else 1
            k += 1
        out.append(O.lower_utf8(s[i:k].encode()))
        i = k
    return out


def engine_tokens(b: bytes):
    from tfidf_amd._lib import UnsupportedInput
    from tfidf_amd.engine import analyze
    try:
        return analyze(b)
    except UnsupportedInput as e:
        raise ValueError(str(e))


# representative characters of every class (plus plain separators)
SAMPLES = {
    "ALETTER": "aZéÉßİKΣσжЖअ々", "HEBREW": "אבג", "NUMERIC": "09١٢１", "KATAKANA": "アカーﾀ゛",
    "EXTNUMLET": "_‿", "MIDLETTER": ":·״", "MIDNUMLET": ".’", "MIDNUM": ",;", "SQUOTE": "'",
    "DQUOTE": '"', "EXTEND": "́̈️­", "EXTEND_SA": "ัิ",
    "ZWJ": "‍", "SA": "กขຂ", "HAN": "中文字", "HIRAGANA": "ひらが", "RI": "\U0001F1FA\U0001F1F8",
    "EMOJI": "\U0001F600❤\U0001F468", "OTHER": " \n\t-!(/#€　​",
}
ALPHA = "".join(SAMPLES.values())


def rand_text(rng, n):
    return "".join(rng.choice(ALPHA) for _ in range(n))


def test_sample_chars_have_their_class():
    txt = open(os.path.join(REPO, "oracle", "unicode_props.h")).read()
    assert "UC_NRANGES" in txt
    for k, chars in SAMPLES.items():
        for ch in chars:
            cp = ord(ch)
            got = next((c for c, rs in R.items() if any(a <= cp <= b for a, b in rs)), "OTHER")
            assert got == k, (hex(cp), got, k)


@pytest.mark.parametrize("seed", range(6))
def test_oracle_and_engine_match_jflex_grammar(seed):
    rng = random.Random(seed)
    for _ in range(150):
        s = rand_text(rng, rng.randint(0, 60))
        want = jflex_tokens(s)
        b = s.encode()
        assert O.tokenize(b, force_unicode=True) == want, repr(s)
        assert engine_tokens(b) == want, repr(s)


def test_ascii_fast_path_equals_unicode_rules():
    rng = random.Random(3)
    alpha = "abcXYZ019_:.',;\" -\n\t#*"
    for _ in range(400):
        b = "".join(rng.choice(alpha) for _ in range(rng.randint(0, 80))).encode()
        assert O.tokenize(b) == O.tokenize(b, force_unicode=True), b
        assert engine_tokens(b) == O.tokenize(b), b


CASES = [
    ("it’s a “quoted” naïve CAFÉ", ["it’s", "a", "quoted", "naïve", "café"]),
    ("İSTANBUL Kelvin ΣΑΣ", ["istanbul", "kelvin", "σασ"]),       # simple (not full) lower-casing
    ("中文 ひらがな カタカナ_abc", ["中", "文", "ひ", "ら", "が", "な", "カタカナ_abc"]),
    ("ภาษาไทย ok", ["ภาษาไทย", "ok"]),
    (" ัก", ["ัก"]),                        # orphan SA mark starts an SA run
    ("_ั ", ["ั"]),                           # ENL run fails; its SA mark is scanned
    ("א\"ב א' א'1", ['א"ב', "א'", "א'1"]),              # WB7a/b/c + Hgrp concatenation
    ("x́y a.́b", ["x́y", "a.́b"]),  # WB4 inside tokens
    ("😀👍🏽 👨‍👩‍👧 🇺🇸🇫", ["😀", "👍🏽", "👨‍👩‍👧", "🇺🇸"]),
    ("１２３ ١٢٫٣ 1.5", ["１２３", "١٢٫٣", "1.5"]),       # U+066B is WB Numeric
    ("\ufeffbom", ["bom"]),                                   # leading Format char (BOM): skipped
]


@pytest.mark.parametrize("text,want", CASES)
def test_cases(text, want):
    w = [t.encode() for t in want]
    assert jflex_tokens(text) == w
    assert O.tokenize(text.encode()) == w
    assert engine_tokens(text.encode()) == w


def test_chop_counts_utf16_units():
    s = "é" * 300 + " " + "a" * 254 + "\U00010400" * 3
    want = jflex_tokens(s)
    assert [len(t.decode()) for t in want][:2] == [255, 45]
    assert O.tokenize(s.encode()) == want
    assert engine_tokens(s.encode()) == want


@pytest.mark.parametrize("bad", [b"\xc0\x80", b"\xed\xa0\x80", b"\xe2\x82", b"\xf5\x80\x80\x80", b"a\xffb",
                                 b"\xf4\x90\x80\x80", b"\xe0\x80\xaf"])
def test_malformed_utf8_rejected(bad):
    with pytest.raises(ValueError):
        O.tokenize(bad)
    with pytest.raises(ValueError):
        engine_tokens(bad)


def test_query_terms_unicode_and_ideographic_space():
    got = O.query_terms("Café　café ÉCOLE".encode())
    assert got == [("café".encode(), 2.0), ("école".encode(), 1.0)]
