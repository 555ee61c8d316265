"""Node-level failure semantics (round-4 advisor findings; include/tfidf.h
"process model (2)"): a rank that cannot serve a search still takes part in
its first collective, so no rank waits for ever —

* GLOBAL searches fail on every rank together: an index re-committed since the
  last GLOBAL exchange (its df / docCount would be shard-local), or two ranks
  whose doc ranges overlap (their merge keys would collide);
* SHARD searches merge the healthy ranks' hits and name the skipped rank
  (Leader.start skips a failed worker, Leader.java:67-69), e.g. a shard
  re-committed after its name table was built.

Every call runs under a thread timeout: a hang is a failure, not a stuck suite.
"""
import threading

import pytest

import multirank as M
from tfidf_amd import _lib as L
from tfidf_amd import distributed as D
from tfidf_amd.engine import ShardIndex

pytestmark = pytest.mark.gpu


def run_ranks(fns, timeout=60):
    """fns[r]() on one thread per rank; returns per-rank (result, exception)."""
    out = [None] * len(fns)

    def body(r):
        try:
            out[r] = (fns[r](), None)
        except Exception as e:            # noqa: BLE001 - reported per rank
            out[r] = (None, e)

    th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
    assert not any(t.is_alive() for t in th), "a rank is still waiting in a collective"
    return out


def _ranks(world, bases=None):
    texts, names = M.corpus()
    comms = D.Comm.inproc(world)
    idx, ads = [], []
    for r in range(world):
        lo, hi = D.shard_range(M.N_DOCS, r, world)
        ix = ShardIndex(device=0)
        ix.add_documents(texts[lo:hi], names[lo:hi])
        ix.commit()
        idx.append(ix)
        ads.append(D.DistShard(ix, comms[r], doc_base=lo if bases is None else bases[r]))
    return comms, idx, ads


def _close(comms, idx):
    for c in comms:
        c.close()
    for i in idx:
        i.close()


def _code(res):
    return [e.code if isinstance(e, L.TfidfError) else ("ok" if e is None else repr(e)) for _, e in res]


def test_global_search_after_a_local_recommit_fails_on_every_rank():
    comms, idx, ads = _ranks(2)
    res = run_ranks([lambda a=a: a.global_commit() for a in ads])
    assert _code(res) == ["ok", "ok"]
    q = M.QUERIES[0]
    res = run_ranks([lambda a=a: a.search(q, M.K) for a in ads])
    assert _code(res) == ["ok", "ok"] and res[0][0] == res[1][0]
    idx[1].commit()                                   # rank 1: local statistics again
    for call in (lambda a: a.search(q, M.K), lambda a: a.search(q, 0), lambda a: a.search_batch(M.QUERIES[:4], 5)):
        res = run_ranks([lambda a=a: call(a) for a in ads])
        assert _code(res) == [L.E_STATE, L.E_STATE], res
    res = run_ranks([lambda a=a: a.global_commit() for a in ads])   # exchange again: serving again
    res = run_ranks([lambda a=a: a.search(q, M.K) for a in ads])
    want = M.expected()["topk"][0]
    assert [r[0] for r in res] == [[(d, float(s)) for d, s in want]] * 2
    _close(comms, idx)


def test_global_search_with_overlapping_doc_ranges_fails_on_every_rank():
    comms, idx, ads = _ranks(2, bases=[0, 0])
    run_ranks([lambda a=a: a.global_commit() for a in ads])
    for k in (M.K, 0):
        res = run_ranks([lambda a=a: a.search(M.QUERIES[0], k) for a in ads])
        assert _code(res) == [L.E_INVALID_ARG, L.E_INVALID_ARG], res
    _close(comms, idx)


def test_uncommitted_rank_fails_global_commit_on_every_rank():
    comms, idx, ads = _ranks(2)
    texts, names = M.corpus()
    fresh = ShardIndex(device=0)                      # rank 1 never committed
    ads[1] = D.DistShard(fresh, comms[1], doc_base=ads[1].doc_base)
    res = run_ranks([lambda a=a: a.global_commit() for a in ads])
    assert _code(res) == [L.E_STATE, L.E_STATE], res
    res = run_ranks([lambda a=a: a.search(M.QUERIES[0], M.K) for a in ads])
    assert _code(res) == [L.E_STATE, L.E_STATE], res
    fresh.close()
    _close(comms, idx)


@pytest.mark.parametrize("skip", [0, 1, 2])
def test_shard_search_skips_a_stale_rank(skip):
    """SPMD SHARD mode, 3 ranks: rank `skip` re-committed after the name
    table -> the other two ranks' Leader merge, on every rank, with the
    skipped rank reported."""
    comms, idx, ads = _ranks(3)
    run_ranks([lambda a=a: a.shard_commit() for a in ads])
    idx[skip].commit()
    want = M.expected_shard(3, skip=(skip,))
    for q, w in zip(M.QUERIES, want):
        res = run_ranks([lambda a=a: (a.shard_search(q), a.last_failed()) for a in ads])
        assert _code(res) == ["ok"] * 3
        for (got, failed), _ in res:
            assert [n for n, _ in got] == [n for n, _ in w]
            assert [s for _, s in got] == [s for _, s in w]
            if q not in M.QUERIES[-2:]:                # a query that does not parse fails before any exchange
                assert failed == 1 << skip
    _close(comms, idx)


def test_node_shard_mode_skips_a_recommitted_shard():
    """tfidf_node (SHARD): a shard committed through its own handle is skipped
    (tfidf_node_last_failed); tfidf_node_commit makes it serve again."""
    n = M_node(3, L.STATS_SHARD)
    L.check(L.load().tfidf_commit(n.shard(1)))
    want = M.expected_shard(3, skip=(1,))
    for q, w in zip(M.QUERIES, want):
        got = n.search_names(q)
        assert [nm for nm, _ in got] == [nm for nm, _ in w]
        assert [s for _, s in got] == [s for _, s in w]
        if q not in M.QUERIES[-2:]:
            assert n.last_failed() == 0b10
    n.commit()
    full = M.expected_shard(3)
    for q, w in zip(M.QUERIES[:4], full):
        assert n.search_names(q) == w
        assert n.last_failed() == 0
    n.close()


def test_node_global_mode_recommitted_shard_fails_then_recovers():
    n = M_node(2, L.STATS_GLOBAL)
    L.check(L.load().tfidf_commit(n.shard(1)))
    with pytest.raises(L.TfidfError) as e:
        n.search(M.QUERIES[0], M.K)
    assert e.value.code == L.E_STATE
    with pytest.raises(L.TfidfError):
        n.search_batch(M.QUERIES[:4], 5)
    n.commit()
    want = M.expected()["topk"][0]
    assert n.search(M.QUERIES[0], M.K) == [(d, float(s)) for d, s in want]
    n.close()


def M_node(shards, mode):
    texts, names = M.corpus()
    n = D.Node(devices=[0] * shards, stats_mode=mode)
    n.add_documents(texts, names)
    n.commit()
    return n
