"""The generated Unicode classes checked against an independent source.

Product (csrc/unicode_tables.h) and oracle (oracle/unicode_props.h) take their
Word_Break classes from one generator (tools/gen_unicode_tables.py: ICU 70
values of the code points assigned in Unicode 9.0), so the GPU-vs-oracle
parity tests cannot catch a wrong class.  The `regex` module carries its own
Unicode database (a later Unicode version); this test compares every code
point the generator gives a Word_Break-derived class with regex's
`\\p{Word_Break=...}`.  Allowed differences, each explained:
* Format folds into Extend (the grammar's `Extend | Format` classes);
* Word_Break values changed after Unicode 9.0 for a few code points
  (U+0600-0605 and U+0890-0891 Format -> Numeric, U+070F and U+110BD/U+110CD
  Format -> ALetter / Numeric-adjacent changes; U+FE10/U+FE14 MidNum -> Other);
* the grammar's own classes (Han, Hiragana, SA and its marks, emoji) that
  Word_Break does not name.
Code points the generator leaves OTHER but regex classes (characters assigned
after Unicode 9.0) are counted, not asserted: the image has no Unicode Age
table to tell them from omissions.
"""
import collections
import os
import re

import pytest

regex = pytest.importorskip("regex")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = ["OTHER", "ALETTER", "HEBREW", "NUMERIC", "KATAKANA", "EXTNUMLET", "MIDLETTER", "MIDNUMLET",
           "MIDNUM", "SQUOTE", "DQUOTE", "EXTEND", "EXTEND_SA", "ZWJ", "SA", "HAN", "HIRAGANA", "RI", "EMOJI"]
WB_OF = {"ALETTER": {"ALetter"}, "HEBREW": {"Hebrew_Letter"}, "NUMERIC": {"Numeric"}, "KATAKANA": {"Katakana"},
         "EXTNUMLET": {"ExtendNumLet"}, "MIDLETTER": {"MidLetter"}, "MIDNUMLET": {"MidNumLet"}, "MIDNUM": {"MidNum"},
         "SQUOTE": {"Single_Quote"}, "DQUOTE": {"Double_Quote"}, "EXTEND": {"Extend", "Format"},
         "EXTEND_SA": {"Extend"}, "ZWJ": {"ZWJ"}, "RI": {"Regional_Indicator"}}
# Word_Break changes after Unicode 9.0 (code point: value in regex's later database)
CHANGED = {0x600: "Numeric", 0x601: "Numeric", 0x602: "Numeric", 0x603: "Numeric", 0x604: "Numeric",
           0x605: "Numeric", 0x6DD: "Numeric", 0x70F: "ALetter", 0x8E2: "Numeric", 0x110BD: "Numeric",
           0x110CD: "Numeric", 0xFE10: "Other", 0xFE14: "Other", 0xFE13: "Other"}
WB = ["ALetter", "Hebrew_Letter", "Numeric", "Katakana", "ExtendNumLet", "MidLetter", "MidNumLet", "MidNum",
      "Single_Quote", "Double_Quote", "Extend", "Format", "ZWJ", "Regional_Indicator"]


def generated_classes():
    txt = open(os.path.join(REPO, "oracle", "unicode_props.h")).read()
    body = txt[txt.index("uc_ranges"):txt.index("UC_NRANGES")]
    out = {}
    for a, b, k in re.findall(r"\{0x([0-9A-F]+), 0x([0-9A-F]+), (\d+)\}", body):
        for c in range(int(a, 16), int(b, 16) + 1):
            out[c] = CLASSES[int(k)]
    return out


def test_generated_word_break_classes_match_an_independent_database():
    gen = generated_classes()
    big = regex.compile("|".join(r"(?P<%s>\p{Word_Break=%s})" % (w, w) for w in WB))
    bad, later = [], collections.Counter()
    for c in range(0x110000):
        if 0xD800 <= c <= 0xDFFF:
            continue
        m = big.match(chr(c))
        w = m.lastgroup if m else "Other"
        g = gen.get(c, "OTHER")
        if g in WB_OF:
            if w not in WB_OF[g] and CHANGED.get(c) != w:
                bad.append((hex(c), g, w))
        elif g == "OTHER" and w != "Other" and CHANGED.get(c) != w:
            later[w] += 1                                    # assigned after 9.0 (or an omission)
    assert not bad, bad[:40]
    # the bulk of the letters the generator classes must be regex's ALetter
    assert sum(1 for g in gen.values() if g == "ALETTER") > 25000
    print("classed by regex, OTHER in the 9.0 tables:", dict(later))


def test_prose_characters_have_the_classes_the_wave_rules_assume():
    """The characters round 6's prose rules rely on, by regex's database."""
    gen = generated_classes()
    wb = lambda ch: next(w for w in WB + ["Other"] if w == "Other" or regex.match(r"\p{Word_Break=%s}" % w, ch))
    for ch in "’‘․":
        assert wb(ch) == "MidNumLet" and gen[ord(ch)] == "MIDNUMLET", ch
    for ch in "·‧":
        assert wb(ch) == "MidLetter" and gen[ord(ch)] == "MIDLETTER", ch
    for ch in " “”—–…«»":
        assert wb(ch) == "Other" and gen.get(ord(ch), "OTHER") == "OTHER", ch
    for ch in "ÉÖÇΣЯéöçσя":
        assert wb(ch) == "ALetter" and gen[ord(ch)] == "ALETTER", ch
