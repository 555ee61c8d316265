"""Rank bodies of the multi-process GPU tests of the node-level orchestration
(libtfidf's tfidf_dist_*, csrc/tfidf_dist.hip, through tfidf_amd/distributed.py):
every rank's ShardIndex on cuda:0, the library's collectives routed through a
callback communicator over the gloo group (RCCL needs one GPU per rank; the
8-GPU RCCL run is the driver's).  Rank 0 writes the results to JSON; the
parent test compares them with single-index (GLOBAL) and per-worker +
Leader-merge (SHARD) oracle results.  The same checks run over the
single-process node (tfidf_node_*, test_gpu_node.py).
"""
import json
import os
import socket

import numpy as np
import torch
import torch.distributed as dist

from oracle import oracle as O
from tfidf_amd import distributed as D
from tfidf_amd import synth

N_DOCS = 1200
K = 25


def corpus():
    """Texts + document names; names repeat across ranks (Leader sums them)
    but never within one rank's contiguous shard (2 or 3 ranks)."""
    texts = synth.corpus(N_DOCS, V=6000, len_min=20, len_max=150)
    names = [b"f%05d.txt" % (i % 700) for i in range(N_DOCS)]
    return texts, names


# the last two do not parse (dangling operator, nothing but an operator):
# Worker.processDocuments answers [] and the Leader merges nothing
QUERIES = synth.queries(12, lo=1, hi=1500) + [b"aaaa", b"aaab aaac", b"aaab AND aaac", b"aaaa NOT aaab",
                                              b"aaab AND", b"OR"]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_queries(search, search_batch, shard_search):
    """The result set every form of the orchestration is checked on."""
    res = {}
    res["topk"] = [[[d, float(s)] for d, s in search(q, K)] for q in QUERIES]
    res["all"] = [[[d, float(s)] for d, s in search(q, 0)] for q in QUERIES[:6] + QUERIES[-2:]]
    bd, bs, bc = search_batch(QUERIES, K)
    res["batch"] = [[[int(bd[i, j]), float(bs[i, j])] for j in range(int(bc[i]))] for i in range(len(QUERIES))]
    return res


def run_rank(rank, world, port, kind, out_path):
    from tfidf_amd.engine import ShardIndex
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    texts, names = corpus()
    lo, hi = D.shard_range(N_DOCS, rank, world)
    torch.cuda.set_device(0)
    idx = ShardIndex(device=0)
    idx.add_documents(texts[lo:hi], names[lo:hi])
    idx.commit()
    comm = D.Comm.from_group(transport="callback")
    ad = D.DistShard(idx, comm, doc_base=lo)
    res = {}
    # SHARD mode (the reference's N workers): own statistics, Leader merge by name
    ad.shard_commit()
    res["shard"] = [[[n.hex(), s] for n, s in ad.shard_search(q)] for q in QUERIES]
    # GLOBAL mode (1-worker semantics)
    nv, dc, ttf = ad.global_commit(vocab_size=True)
    res.update(n_vocab=nv, dc=dc, ttf=ttf)
    res.update(run_queries(ad.search, ad.search_batch, None))
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()
    idx.close()


def expected():
    """Single-index (GLOBAL) and per-worker + Leader (SHARD) oracle results."""
    texts, names = corpus()
    one = O.OracleIndex()
    for i, t in enumerate(texts):
        one.add_doc(str(i).encode(), t)
    one.commit()
    out = {"dc": one.doc_count, "ttf": one.sum_ttf, "n_vocab": one.num_terms}

    def search(ix, q, k):
        try:
            return ix.search(q, k)
        except O.QuerySyntaxError:
            return []

    out["topk"] = [search(one, q, K) for q in QUERIES]
    out["all"] = [search(one, q, 0) for q in QUERIES[:6] + QUERIES[-2:]]
    one.close()
    return out


def expected_shard(world, skip=()):
    """Per-worker oracles + the Leader merge; ranks in `skip` are failed
    workers whose responses the Leader never sees (Leader.java:67-69)."""
    texts, names = corpus()
    workers = []
    for r in range(world):
        if r in skip:
            continue
        lo, hi = D.shard_range(N_DOCS, r, world)
        o = O.OracleIndex()
        for n, t in zip(names[lo:hi], texts[lo:hi]):
            o.add_doc(n, t)
        o.commit()
        workers.append(o)
    out = []
    for q in QUERIES:
        resp = []
        for o in workers:
            try:
                resp.append([(o.doc_key(d), float(s)) for d, s in o.search(q, 0)])
            except O.QuerySyntaxError:
                resp.append([])
        out.append(O.leader_merge(resp))
    for o in workers:
        o.close()
    return out


def check(res, world):
    want = expected()
    assert (res["dc"], res["ttf"], res["n_vocab"]) == (want["dc"], want["ttf"], want["n_vocab"])

    def same(got, exp):
        assert [d for d, _ in got] == [d for d, _ in exp]
        assert [np.float32(s) for _, s in got] == [np.float32(s) for _, s in exp]

    for q, a, b, w in zip(QUERIES, res["topk"], res["batch"], want["topk"]):
        same(a, w)
        same(b, w)
    for a, w in zip(res["all"], want["all"]):
        same(a, w)
    for got, w in zip(res["shard"], expected_shard(world)):
        assert [bytes.fromhex(n) for n, _ in got] == [n for n, _ in w]
        assert [s for _, s in got] == [s for _, s in w]          # double sums, exactly


# ---------------------------------------------------------------------------
# Hash-seed agreement (GLOBAL statistics match hashed term keys across shards:
# a shard that met a collision rebuilt under a later seed, and the others must
# follow it).  Corpus with hashed keys: terms over 16 bytes and non-ASCII terms.

def seed_corpus():
    rng = np.random.default_rng(11)
    base = synth.corpus(400, V=3000, len_min=10, len_max=60)
    longw = [bytes(rng.integers(97, 123, int(rng.integers(17, 21))).astype(np.uint8)) for _ in range(40)]
    # (the last two: non-ASCII terms over 14 bytes, so hashed keys — of equal
    # length, so they collide under TFIDF_TEST_WEAK_HASH; shorter ones are exact)
    uni = [w.encode() for w in ("café", "naïve", "über", "façade", "señor", "ångström", "smörgåsbord",
                                 "crème", "brûlée", "jalapeño", "Ελλάδα", "москва", "日本語",
                                 "übernationalität", "übernationalitát")]
    texts = []
    for i, t in enumerate(base):
        extra = [longw[int(j)] for j in rng.integers(0, len(longw), 3)] + [uni[int(j)] for j in
                                                                           rng.integers(0, len(uni), 2)]
        texts.append(t + b" " + b" ".join(extra))
    names = [b"s%04d.txt" % i for i in range(len(texts))]
    return texts, names


SEED_QUERIES = [b"caf\xc3\xa9 aaab", b"na\xc3\xafve \xc3\xbcber", b"aaaa"]


def _seed_queries():
    texts, _ = seed_corpus()
    toks = texts[5].split(b" ")
    return SEED_QUERIES + [b" ".join(toks[-5:-2]), toks[-4]]


def run_rank_seed(rank, world, port, kind, out_path):
    """The real engine, shard 1 (only) under TFIDF_TEST_WEAK_HASH (every pair
    of equal-length hashed keys collides: its commit moves to attempt 1); the
    library's GLOBAL exchange has the other shards re-commit under it."""
    from tfidf_amd.engine import ShardIndex
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    texts, names = seed_corpus()
    lo, hi = D.shard_range(len(texts), rank, world)
    torch.cuda.set_device(0)
    if rank == 1:
        os.environ["TFIDF_TEST_WEAK_HASH"] = "1"
    idx = ShardIndex(device=0)
    idx.add_documents(texts[lo:hi], names[lo:hi])
    idx.commit()
    os.environ.pop("TFIDF_TEST_WEAK_HASH", None)
    before = int(idx.stats()["hash_rebuilds"])
    comm = D.Comm.from_group(transport="callback")
    ad = D.DistShard(idx, comm, doc_base=lo)
    nv, dc, ttf = ad.global_commit(vocab_size=True)
    res = {"before": before, "after": int(idx.stats()["hash_rebuilds"]), "n_vocab": nv, "dc": dc, "ttf": ttf,
           "topk": [[[d, float(s)] for d, s in ad.search(q, K)] for q in _seed_queries()]}
    with open("%s.%d" % (out_path, rank), "w") as f:
        json.dump(res, f)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()
    idx.close()


def check_seed(out_path, world):
    res = [json.load(open("%s.%d" % (out_path, r))) for r in range(world)]
    texts, _ = seed_corpus()
    one = O.OracleIndex()
    for i, t in enumerate(texts):
        one.add_doc(str(i).encode(), t)
    one.commit()
    want = [one.search(q, K) for q in _seed_queries()]
    assert all(w for w in want)
    for r in res:
        assert (r["n_vocab"], r["dc"], r["ttf"]) == (one.num_terms, one.doc_count, one.sum_ttf)
        assert len({x["after"] for x in res}) == 1
        for got, w in zip(r["topk"], want):
            assert [d for d, _ in got] == [d for d, _ in w]
            assert [np.float32(s) for _, s in got] == [np.float32(s) for _, s in w]
    one.close()
    return res
