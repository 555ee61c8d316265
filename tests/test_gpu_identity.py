"""Exact term identity for hashed keys (terms of more than 16 bytes, and
non-ASCII terms of more than 14; shorter non-ASCII terms have exact keys
since round 5): the engine never lets two different terms share a
key.  Every merge under a hashed key compares the lower-cased strings (the
per-document tables of the Unicode wave path and of the long path, and the
global dictionary through each slot's reference occurrence); a mismatch makes
the commit start over with another hash seed.

TFIDF_TEST_WEAK_HASH=1 starts the commit from a seed under which EVERY two
hashed keys of equal byte length collide, so these corpora exercise the
detection on each path and the rebuild; the results must still equal the CPU
oracle (which keys terms by their strings), and tfidf_doc_terms returns the
real strings of hashed terms.
"""
import random

import pytest

from oracle import oracle as O
from tfidf_amd.engine import ShardIndex
from test_gpu_parity import assert_hits_equal

pytestmark = pytest.mark.gpu

LONG = [b"internationalisationX", b"internationalisationY", b"internationalisationZ"]   # 21 bytes, one prefix
UNI = ["café", "cafè", "CAFÉ", "naïve", "naîve", "ĳssel", "straße", "Straße", "über", "ÜBER", "öber",
       "übernationalität", "übernationalitát"]   # (> 14 bytes: hashed keys, colliding under the weak seed)


def corpus(seed, n=300):
    rng = random.Random(seed)
    texts = []
    for i in range(n):
        words = []
        for _ in range(rng.randint(3, 40)):
            r = rng.random()
            if r < 0.25:
                words.append(rng.choice(LONG))
            elif r < 0.5:
                words.append(rng.choice(UNI).encode())
            else:
                words.append(rng.choice([b"alpha", b"beta", b"gamma", b"delta"]))
        texts.append(b" ".join(words))
    # a long-path document (> 4 KB window) and a book-sized one, both mixed
    texts.append(b" ".join(rng.choice(LONG + [u.encode() for u in UNI]) for _ in range(1500)))
    texts.append(b" ".join(rng.choice(LONG + [b"plain", b"words"]) for _ in range(6000)))
    return texts


def check(texts, expect_rebuilds):
    g = ShardIndex()
    g.add_documents(texts)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    st = g.stats()
    assert st["hash_rebuilds"] == expect_rebuilds
    assert (st["num_terms"], st["nnz"], st["sum_ttf"]) == (o.num_terms, sum(o.vocab().values()), o.sum_ttf)
    for d in range(len(texts)):
        assert g.doc_terms(d) == o.doc_terms(d), d
    for t, df in o.vocab().items():                                # every term, exact strings
        assert g.df(t)[0] == df, t
    for q in LONG + [u.encode() for u in UNI] + [b"cafe", b"internationalisation"]:
        assert_hits_equal(g.search(q, 0), o.search(q, 0))
    g.close()
    o.close()
    return st


def test_hashed_terms_exact_without_collisions():
    st = check(corpus(1), 0)
    assert st["hash_seed"] == 0


def test_forced_collisions_are_detected_and_rebuilt(monkeypatch):
    monkeypatch.setenv("TFIDF_TEST_WEAK_HASH", "1")
    st = check(corpus(2), 1)
    assert st["hash_seed"] == 1
