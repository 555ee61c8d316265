"""GPU parity of the wave tokenizer's XCD-contiguous unit ranges (workgroup b
takes units from the eighth b mod 8 of the corpus, kernels_index.hip
k_tokenize_wave) against the CPU oracle: corpora with at least as many units
as the persistent grid has workgroups, so the mapping is the one that runs
(the small parity corpora take the plain grid stride).  Single documents per
window (cfg-2 shape), packed short documents (cfg-5 shape), and the cfg-2
shape with every third document non-ASCII (flagged per document for the
Unicode document wave, which reads the flags 64 at a time across the grid)."""
import random

import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

pytestmark = pytest.mark.gpu


def _non_ascii_every_third(texts):
    """Every third document: the first two letters of its first word become
    U+00E9 / U+00C9 (same byte length), alternating, so both the lower-cased
    and the upper-case form reach the Unicode path."""
    out = []
    for i, t in enumerate(texts):
        if i % 3 == 0 and len(t) >= 2 and t[:2].isalpha():
            t = (b"\xc3\xa9" if i % 2 else b"\xc3\x89") + t[2:]
        out.append(t)
    return out


@pytest.mark.parametrize("shape", ["single", "packed", "unicode"])
def test_xcd_contiguous_units_match_oracle(shape):
    if shape == "single":
        texts = synth.corpus(20000, V=50000, len_min=300, len_max=500)
    elif shape == "unicode":
        texts = _non_ascii_every_third(synth.corpus(20000, V=50000, len_min=300, len_max=500))
    else:
        texts = synth.corpus(25000, V=60000, len_min=30, len_max=70)
    g = ShardIndex(vocab_capacity_log2=18)
    g.add_documents(texts)
    g.commit()
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    try:
        s = g.stats()
        if shape == "packed":
            assert s["pack_docs"] > 1
        if shape == "unicode":
            assert s["unicode_docs"] == sum(1 for t in texts if max(t) >= 0x80)
        assert (s["doc_count"], s["sum_ttf"], s["num_terms"]) == (o.doc_count, o.sum_ttf, o.num_terms)
        rng = random.Random(11)
        n = len(texts)
        # documents from every eighth of the corpus (every XCD's range) and the range edges
        docs = sorted(set(rng.sample(range(n), 400) + [0, n - 1] + [n * x // 8 for x in range(8)] +
                          [n * x // 8 - 1 for x in range(1, 8)]))
        for d in docs:
            assert g.doc_terms(d) == o.doc_terms(d)
            assert g.doc_len(d) == (o.doc_len(d), o.doc_norm(d))
        vocab = o.vocab()
        for t in rng.sample(sorted(vocab), 300):
            assert g.df(t)[0] == vocab[t]
        for q in synth.queries(12, lo=1, hi=3000):
            got, want = g.search(q, 10), o.search(q, 10)
            assert [d for d, _ in got] == [d for d, _ in want]
            assert [float(x) for _, x in got] == [float(x) for _, x in want]
    finally:
        g.close()
        o.close()
