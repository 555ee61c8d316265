"""Cross-check the oracle's UAX#29 local-rule tokenizer against an independent
restatement of Lucene 9.8.0's JFlex grammar (StandardTokenizerImpl.jflex,
WORD_TYPE / NUMERIC_TYPE rules, ASCII subset) evaluated by longest match.

The two formulations are structurally different (per-position break rules vs a
maximal-munch regular grammar), so agreement on random strings over the
joiner alphabet is evidence that the ASCII tokenizer semantics are right.
"""
import re

import pytest
from hypothesis import given, settings, strategies as st

from oracle import oracle as O

# {ExtendNumLetEx} = '_'; {MidLetterEx} = MidLetter | MidNumLet | Single_Quote = [:.'];
# {MidNumericEx} = MidNum | MidNumLet | Single_Quote = [,;.']
LETTER_RUN = r"[A-Za-z](?:(?:_*|[:.'])[A-Za-z])*"
NUMERIC_RUN = r"[0-9](?:(?:_*|[,;.'])[0-9])*"
RUNS = r"(?:%s|%s)+" % (LETTER_RUN, NUMERIC_RUN)
WORD = re.compile(r"_*%s(?:_+%s)*_*" % (RUNS, RUNS))


def jflex_tokens(s: str):
    out = []
    i = 0
    n = len(s)
    while i < n:
        best = 0
        for j in range(n, i, -1):           # longest match first
            if WORD.fullmatch(s, i, j):
                best = j - i
                break
        if best:
            out.append(s[i:i + best].lower())
            i += best
        else:
            i += 1                            # [^] rule: skip one char
    return out


CASES = {
    "Hello World": ["hello", "world"],
    "U.S.A.": ["u.s.a"],
    "3,14 1.2.3": ["3,14", "1.2.3"],
    "don't a:b": ["don't", "a:b"],
    "a.1 10:30 e-mail a..b": ["a", "1", "10", "30", "e", "mail", "a", "b"],
    "___ _x_ a__1 1_a": ["_x_", "a__1", "1_a"],
    "a1.2 1a.b a1:b ab.1": ["a1.2", "1a.b", "a1", "b", "ab", "1"],
    "fast food .": ["fast", "food"],
    "best wireless earbuds 2024": ["best", "wireless", "earbuds", "2024"],
    "'quoted' x'": ["quoted", "x"],
    "a_.b a:_b 1'2": ["a_", "b", "a", "_b", "1'2"],
}


@pytest.mark.parametrize("text,want", list(CASES.items()))
def test_known_cases(text, want):
    assert [t.decode() for t in O.tokenize(text.encode())] == want
    assert jflex_tokens(text) == want


@settings(max_examples=400, deadline=None)
@given(st.text(alphabet="aZq09_:.',; -\n", max_size=40))
def test_local_rules_equal_jflex_longest_match(s):
    assert [t.decode() for t in O.tokenize(s.encode())] == jflex_tokens(s)


def test_long_token_chopped_at_255():
    s = b"a" * 600
    toks = O.tokenize(s)
    assert [len(t) for t in toks] == [255, 255, 90]


def test_malformed_utf8_rejected():
    with pytest.raises(ValueError):
        O.tokenize(b"caf\xe9")          # Latin-1, not UTF-8: Files.readString would throw
    assert O.tokenize("café".encode()) == ["café".encode()]
