"""All hits (k = 0, searcher.search(q, Integer.MAX_VALUE), Worker.java:230) on
an index of 10 doc blocks: the per-block sorted runs go through the 8-run
group merge (levels 0-2 in one workgroup per group: in LDS when a group holds
<= 8192 hits, else through global memory) and one pairwise merge level.
The group merge is chosen per query (hit bound = sum of the scoring terms'
df); TFIDF_HITS_GROUPS / TFIDF_HITS_PAIRWISE force either path.  Against the
C oracle and path against path; bar: doc ids and float32 score bits identical.
"""
import pytest

from tfidf_amd import synth
from test_gpu_parity import assert_hits_equal, build_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def corpus():
    # 80 k short documents = 10 blocks of 8192; V = 2000: the most frequent
    # terms hit ~60 % of the documents (groups far over the LDS capacity),
    # mid-rank terms a few percent (groups merged in LDS)
    texts = synth.corpus(80_000, V=2000, len_min=2, len_max=12)
    g, o = build_pair(texts)
    yield g, o
    g.close()
    o.close()


QUERIES = (synth.queries(3, n_terms=1, lo=0, hi=3) + synth.queries(4, n_terms=1, lo=20, hi=200) +
           synth.queries(4, n_terms=2, lo=0, hi=400) + synth.queries(3, n_terms=3, lo=500, hi=2000))


@pytest.mark.parametrize("force", [None, "TFIDF_HITS_GROUPS", "TFIDF_HITS_PAIRWISE"])
def test_all_hits_equal_oracle(corpus, monkeypatch, force):
    """Default (group merge chosen per query by its hit bound), forced group
    merge (the frequent terms' groups overflow the LDS: global-memory path)
    and the pairwise levels only."""
    g, o = corpus
    if force:
        monkeypatch.setenv(force, "1")
    big = 0
    for q in QUERIES:
        want = o.search(q, 0)
        big += len(want) > 8 * 8192 * 0.125
        assert_hits_equal(g.search(q, 0), want)
    assert big >= 2                                    # groups over the LDS capacity exist


def test_group_merge_equals_pairwise_levels(corpus, monkeypatch):
    g, _ = corpus
    monkeypatch.setenv("TFIDF_HITS_GROUPS", "1")
    got = [g.search(q, 0) for q in QUERIES]
    monkeypatch.delenv("TFIDF_HITS_GROUPS")
    monkeypatch.setenv("TFIDF_HITS_PAIRWISE", "1")
    ref = [g.search(q, 0) for q in QUERIES]
    assert got == ref
