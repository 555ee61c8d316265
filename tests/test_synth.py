"""Synthetic corpus generator: definition checks on the host generator, and
(GPU) bit-identity of the device generator with it."""
import numpy as np
import pytest

from tfidf_amd import synth
from oracle import oracle as O


def test_word_bijective_base26():
    assert synth.word(1) == b"aaaa"
    assert synth.word(2) == b"aaab"
    assert synth.word(26) == b"aaaz"
    assert synth.word(27) == b"aaba"
    assert synth.word(456976) == b"zzzz"
    assert synth.word(456977) == b"aaaaa"
    ws = [synth.word(r) for r in range(1, 3000)]
    assert len(set(ws)) == len(ws)


def test_doc_lengths_and_separators():
    docs = synth.corpus(50, V=1000, len_min=40, len_max=60)
    for d, t in enumerate(docs):
        toks = t.split()
        assert 40 <= len(toks) <= 60
        assert len(toks) == synth.doc_tokens(synth.SEED, d, 40, 60)
        assert t.endswith(b"\n")
        assert t.count(b"\n") == (len(toks) + 15) // 16
        # every token is one analyzer token (pure lowercase letters)
        assert O.tokenize(t) == toks


def test_zipf_rank_frequencies():
    cdf = synth.zipf_cdf(1000)
    ranks = np.concatenate([synth.doc_ranks(synth.SEED, d, 400, 600, cdf) for d in range(200)])
    counts = np.bincount(ranks, minlength=1001)
    # Zipf s=1: rank 1 about twice rank 2, about 10x rank 10
    assert 1.7 < counts[1] / counts[2] < 2.3
    assert 7 < counts[1] / counts[10] < 13


def test_queries_distinct_midrange():
    qs = synth.queries(100)
    for q in qs:
        ws = q.split()
        assert len(ws) == 3 and len(set(ws)) == 3
        for w in ws:
            assert 4 <= len(w) <= 5


@pytest.mark.gpu
def test_device_generator_bit_identical():
    import ctypes as C
    import torch
    from tfidf_amd import _lib as L
    dc = synth.DeviceCorpus(300, V=5000, len_min=20, len_max=90, doc_base=17)
    try:
        host = synth.corpus(300, V=5000, len_min=20, len_max=90, doc_base=17)
        offs = np.zeros(301, np.uint64)
        text = np.zeros(dc.total_bytes, np.uint8)
        lib = L.load()
        assert dc.total_bytes == sum(len(t) for t in host)
        torch.cuda.synchronize()
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        assert hip.hipMemcpy(offs.ctypes.data, C.c_void_p(dc.d_offsets), 301 * 8, 2) == 0
        assert hip.hipMemcpy(text.ctypes.data, C.c_void_p(dc.d_text), dc.total_bytes, 2) == 0
        assert bytes(text) == b"".join(host)
        assert offs.tolist() == np.concatenate([[0], np.cumsum([len(t) for t in host])]).tolist()
        del lib
    finally:
        dc.free()
