"""The block-major inversion under every launch shape it accepts.

`launch_scatter` (csrc/kernels_index.hip) reads three launch knobs per build:
TFIDF_PART_THREADS (k_scatter_part: 1 024 default, 512, 256 — the round's
document group and its LDS staging scale with the waves per workgroup),
TFIDF_SORT_THREADS (k_scatter_sort: 512 default, 256, 1 024) and
TFIDF_SORT_SPW (sub-range streams per sort workgroup, 4 default).  The
posting order inside a (block, slot) segment is free, so each shape must give
the same index: identical statistics, document frequencies, all-hits lists
and batched top-10 results as the default shape (which tests/test_gpu_parity.py
and tests/test_gpu_fullsize.py hold against the oracle).

The corpus (40 000 cfg-2-style documents, five 8 192-document blocks) has CSR
segments longer than 64 entries (the part pass's per-wave follow-up loads) and
sort streams above the 8 192-entry LDS stage (the scattered-store path).
"""
import numpy as np
import pytest

from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

pytestmark = pytest.mark.gpu

N_DOCS = 40_000
SHAPES = [
    {"TFIDF_PART_THREADS": "512"},
    {"TFIDF_PART_THREADS": "256"},
    {"TFIDF_SORT_THREADS": "256"},
    {"TFIDF_SORT_THREADS": "1024", "TFIDF_SORT_SPW": "1"},
    {"TFIDF_SORT_SPW": "8"},
]


def _snapshot(dc, queries, all_terms, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = ShardIndex()
    try:
        g.add_documents_device(dc.d_text, dc.d_offsets, dc.n_docs, dc.total_bytes)
        g.commit()
        st = g.stats()
        dfs = [g.df(t)[0] for t in all_terms]
        hits = [g.search_all_arrays(t) for t in all_terms]
        docs, scores, counts = g.search_batch(queries, 10)
        return st, dfs, hits, (docs, scores, counts)
    finally:
        g.close()
        for k in env:
            monkeypatch.delenv(k, raising=False)


@pytest.fixture(scope="module")
def corpus():
    dc = synth.DeviceCorpus(N_DOCS)
    yield dc
    dc.free()


def test_inversion_shapes_identical(corpus, monkeypatch):
    queries = synth.queries(300)
    # frequent (ranks 1, 3 — the generator ranks from 1 — in every block's first sub-range stream), middle and rare terms
    all_terms = [synth.word(r) for r in (1, 3, 50, 700, 9000, 60000)]
    base = _snapshot(corpus, queries, all_terms, monkeypatch, {})
    st0, df0, hits0, (d0, s0, c0) = base
    assert st0["doc_count"] == N_DOCS
    assert df0[0] > 8192, "the most frequent term must fill a sort stream past the LDS stage"
    for (docs, scores), df in zip(hits0, df0):
        assert len(docs) == df
    for env in SHAPES:
        st, dfs, hits, (d, s, c) = _snapshot(corpus, queries, all_terms, monkeypatch, env)
        assert st == st0, env
        assert dfs == df0, env
        for (a_doc, a_sc), (b_doc, b_sc) in zip(hits, hits0):
            assert np.array_equal(a_doc, b_doc), env
            assert np.array_equal(a_sc.view(np.int32), b_sc.view(np.int32)), env
        assert np.array_equal(c, c0), env
        assert np.array_equal(d, d0), env
        assert np.array_equal(s.view(np.int32), s0.view(np.int32)), env
