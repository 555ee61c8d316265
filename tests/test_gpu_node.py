"""Process model (1) of the node-level C ABI (tfidf_node_*: one process owns
the shards, a worker thread per shard runs the library's orchestration) and
the built-in RCCL communicator, against the CPU oracle (tests/multirank.py):

* a node of 2 and 3 shards on cuda:0 (a repeated device: the in-process
  transport), GLOBAL mode = the single-index oracle (statistics, top-k, all
  hits, batch), SHARD mode = per-worker oracles + the Leader merge by name;
* a node over device mask 0x1 (ncclCommInitAll, one rank) and a per-rank
  communicator from tfidf_rccl_unique_id / tfidf_comm_init_rccl (world 1):
  the RCCL transport runs the same exchanges;
* global doc id -> document key across shards (Worker.java:235-236).
"""
import ctypes as C

import pytest

import multirank as M
from tfidf_amd import _lib as L
from tfidf_amd import distributed as D

pytestmark = pytest.mark.gpu


def _node(devices, mode, inproc=False):
    texts, names = M.corpus()
    n = D.Node(devices=devices, stats_mode=mode, inproc=inproc)
    n.add_documents(texts, names)
    n.commit()
    return n


@pytest.mark.parametrize("shards", [2, 3])
def test_node_global_equals_oracle(shards):
    n = _node([0] * shards, L.STATS_GLOBAL)
    st = n.stats()
    assert st["transport"] == 2 and st["n_shards"] == shards and st["num_docs"] == M.N_DOCS
    res = {"n_vocab": st["num_terms"], "dc": st["doc_count"], "ttf": st["sum_ttf"], "shard": None}
    res.update(M.run_queries(n.search, n.search_batch, None))
    want = M.expected()
    assert (res["dc"], res["ttf"], res["n_vocab"]) == (want["dc"], want["ttf"], want["n_vocab"])
    for a, b, w in zip(res["topk"], res["batch"], want["topk"]):
        assert a == [[d, float(s)] for d, s in w]
        assert b == [[d, float(s)] for d, s in w]
    for a, w in zip(res["all"], want["all"]):
        assert a == [[d, float(s)] for d, s in w]
    texts, names = M.corpus()
    for d in (0, 399, 400, 401, M.N_DOCS - 1):
        assert n.doc_key(d) == names[d]
    n.close()


@pytest.mark.parametrize("shards", [2, 3])
def test_node_shard_mode_equals_leader_merge(shards):
    n = _node([0] * shards, L.STATS_SHARD)
    want = M.expected_shard(shards)
    for q, w in zip(M.QUERIES, want):
        got = n.search_names(q)
        assert [nm for nm, _ in got] == [nm for nm, _ in w]
        assert [s for _, s in got] == [s for _, s in w]          # double sums, exactly
    n.close()


def unique_names():
    """One shard holds the whole corpus: names must not repeat within it
    (M.corpus() repeats names across the 2- / 3-rank shards; replace-by-key
    would drop documents here)."""
    texts, _ = M.corpus()
    return texts, [b"d%05d.txt" % i for i in range(len(texts))]


def test_node_rccl_one_gpu():
    """Device mask 0x1: the RCCL transport (ncclCommInitAll over one device)."""
    texts, names = unique_names()
    cfg = L.Config()
    lib = L.load()
    L.check(lib.tfidf_config_init(C.byref(cfg)))
    cfg.stats_mode = L.STATS_GLOBAL
    h = C.c_void_p()
    L.check(lib.tfidf_node_create(C.byref(cfg), 1, C.byref(h)))
    n = D.Node.__new__(D.Node)
    n._h = h
    assert n.stats()["transport"] == 1
    n.add_documents(texts, names)
    n.commit()
    want = M.expected()
    for q, w in zip(M.QUERIES, want["topk"]):
        assert n.search(q, M.K) == [(d, float(s)) for d, s in w]
    n.close()


def test_rccl_comm_world1_dist_calls():
    """tfidf_rccl_unique_id + tfidf_comm_init_rccl (world 1): the per-rank
    calls over the built-in RCCL communicator = the single-index oracle."""
    from tfidf_amd.engine import ShardIndex
    lib = L.load()
    uid = (C.c_uint8 * 128)()
    L.check(lib.tfidf_rccl_unique_id(uid))
    h = C.c_void_p()
    L.check(lib.tfidf_comm_init_rccl(uid, 0, 1, 0, C.byref(h)))
    comm = D.Comm(h)
    assert comm.info() == (0, 1, "rccl")
    comm.selftest()
    texts, names = unique_names()
    idx = ShardIndex(device=0)
    idx.add_documents(texts, names)
    idx.commit()
    ad = D.DistShard(idx, comm, doc_base=0)
    nv, dc, ttf = ad.global_commit(vocab_size=True)
    want = M.expected()
    assert (nv, dc, ttf) == (want["n_vocab"], want["dc"], want["ttf"])
    res = M.run_queries(ad.search, ad.search_batch, None)
    for a, b, w in zip(res["topk"], res["batch"], want["topk"]):
        assert a == [[d, float(s)] for d, s in w]
        assert b == [[d, float(s)] for d, s in w]
    assert ad.shard_commit() == len(names)
    for q in M.QUERIES[:6] + M.QUERIES[-2:]:                  # one worker: the Leader map = its own hits by name
        try:
            hits = idx.search(q, 0)
        except L.QuerySyntaxError:
            hits = []
        want = sorted(((names[d], float(s)) for d, s in hits), key=lambda x: x[0])
        assert ad.shard_search(q) == want
    comm.close()
    idx.close()
