"""Rank body shared by the multi-process tests of tfidf_amd/distributed.py
(test_distributed_gloo.py: CPU oracle adapter; test_gpu_multirank.py: the real
HipShardAdapter, every rank's ShardIndex on cuda:0).  Collectives run over
gloo (RCCL needs one GPU per rank).  Rank 0 writes the results to JSON; the
parent test compares them with single-index (GLOBAL) and per-worker +
Leader-merge (SHARD) oracle results.
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
from tfidf_amd.engine import term_key

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


def _keys(docs, scores, base):
    d = (np.asarray(docs, np.uint64) + np.uint64(base)) & np.uint64(0xFFFFFFFF)
    k = (np.asarray(scores, np.float32).view(np.uint32).astype(np.uint64) << np.uint64(32)) | \
        (~d & np.uint64(0xFFFFFFFF))
    return k.view(np.int64)


class OracleShardAdapter:
    """The CPU oracle behind HipShardAdapter's interface (host tensors)."""
    device = torch.device("cpu")
    query_errors = (O.QuerySyntaxError,)

    def __init__(self, texts, names, doc_base):
        self.o = O.OracleIndex()
        for n, t in zip(names, texts):
            self.o.add_doc(n, t)
        self.o.commit()
        self.doc_base = doc_base
        self.names = list(names)

    def local_stats(self):
        return self.o.doc_count, self.o.sum_ttf, self.o.num_docs

    def export_vocab(self):
        vocab = self.o.vocab()
        self.terms = {}
        rows = []
        for t, df in vocab.items():
            lo, hi = term_key(t)
            self.terms[(lo, hi)] = t
            rows.append((hi, lo, df))
        rows.sort()
        keys = np.array([[lo, hi] for hi, lo, _ in rows], np.uint64).reshape(-1, 2)
        df = np.array([d for _, _, d in rows], np.int32)
        self.my_df = {(lo, hi): d for hi, lo, d in rows}
        return torch.from_numpy(keys.view(np.int64).copy()), torch.from_numpy(df)

    def canonicalize(self, all_keys):
        k = all_keys.numpy().view(np.uint64)
        k = k[k[:, 1] != 0]
        order = np.lexsort((k[:, 0], k[:, 1]))
        k = k[order]
        keep = np.ones(len(k), bool)
        keep[1:] = np.any(k[1:] != k[:-1], axis=1)
        self.canon = k[keep]
        self.canon_index = {(int(lo), int(hi)): i for i, (lo, hi) in enumerate(self.canon.tolist())}
        dfc = np.zeros(len(self.canon), np.int32)
        for key, d in self.my_df.items():
            dfc[self.canon_index[key]] = d
        return torch.from_numpy(dfc)

    def import_global(self, dfc, doc_count, sum_ttf):
        dfc = dfc.numpy()
        self.o.set_global_stats(doc_count, sum_ttf,
                                {t: int(dfc[self.canon_index[key]]) for key, t in self.terms.items()})

    @staticmethod
    def _owner(lo, hi, G):
        return ((lo * 0x9E3779B97F4A7C15 ^ hi) & 0xFFFFFFFFFFFFFFFF) % G

    def vocab_partition(self, n_ranks):
        groups = [[] for _ in range(n_ranks)]
        by_owner = [[] for _ in range(n_ranks)]
        for t, df in sorted(self.o.vocab().items()):
            lo, hi = term_key(t)
            r = self._owner(lo, hi, n_ranks)
            groups[r].append((lo, hi, df))
            by_owner[r].append(t)
        self.sent_terms = [t for g in by_owner for t in g]
        rows = [x for g in groups for x in g]
        rec = np.array(rows, np.uint64).reshape(-1, 3).view(np.int64)
        return torch.from_numpy(rec.copy()), torch.tensor([len(g) for g in groups], dtype=torch.int64)

    def vocab_reduce(self, records):
        r = records.numpy().view(np.uint64)
        tot = {}
        for lo, hi, df in r.tolist():
            tot[(lo, hi)] = tot.get((lo, hi), 0) + df
        ans = np.array([tot[(lo, hi)] for lo, hi, _ in r.tolist()], np.int32)
        return torch.from_numpy(ans), torch.tensor([len(tot)], dtype=torch.int64)

    def import_global_df(self, gdf, doc_count, sum_ttf):
        self.o.set_global_stats(doc_count, sum_ttf, {t: int(d) for t, d in zip(self.sent_terms, gdf.tolist())})

    def topk_keys(self, queries, k):
        out = np.zeros((len(queries), k), np.int64)
        for i, q in enumerate(queries):
            try:
                hits = self.o.search(q, k)
            except O.QuerySyntaxError:
                hits = []
            if hits:
                out[i, :len(hits)] = _keys([d for d, _ in hits], [s for _, s in hits], self.doc_base)
        return torch.from_numpy(out)

    def all_keys(self, query, doc_base=None):
        hits = self.o.search(query, 0)
        base = self.doc_base if doc_base is None else doc_base
        return torch.from_numpy(_keys([d for d, _ in hits], [s for _, s in hits], base).copy())

    def doc_names(self):
        blob = np.frombuffer(b"".join(self.names), np.uint8).copy()
        offs = np.zeros(len(self.names) + 1, np.uint64)
        offs[1:] = np.cumsum([len(n) for n in self.names], dtype=np.uint64)
        return blob, offs


def run_rank(rank, world, port, kind, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    texts, names = corpus()
    lo, hi = D.shard_range(N_DOCS, rank, world)
    idx = None
    if kind == "hip":
        from tfidf_amd.engine import ShardIndex
        torch.cuda.set_device(0)
        idx = ShardIndex(device=0)
        idx.add_documents(texts[lo:hi], names[lo:hi])
        idx.commit()
        ad = D.HipShardAdapter(idx, torch.device("cuda", 0), doc_base=lo)
    else:
        ad = OracleShardAdapter(texts[lo:hi], names[lo:hi], lo)
    res = {}
    # SHARD mode (the reference's N workers): own statistics, Leader merge by name
    sn = D.shard_commit(ad)
    res["shard"] = [[[n.hex(), s] for n, s in D.shard_search(ad, sn, q)] for q in QUERIES]
    # GLOBAL mode (1-worker semantics)
    nv, dc, ttf = D.global_commit(ad, vocab_size=True)
    res.update(n_vocab=nv, dc=dc, ttf=ttf)
    res["topk"] = [[[d, float(s)] for d, s in D.global_search(ad, q, K)] for q in QUERIES]
    res["all"] = [[[d, float(s)] for d, s in D.global_search(ad, q, 0)] for q in QUERIES[:6] + QUERIES[-2:]]
    bd, bs, bc = D.global_search_batch(ad, QUERIES, K)
    res["batch"] = [[[int(bd[i, j]), float(bs[i, j])] for j in range(int(bc[i]))] for i in range(len(QUERIES))]
    # the canonical (all-gather + sorted union) form must agree
    n2, dc2, ttf2 = D.global_commit_canonical(ad)
    res["canonical"] = [n2, dc2, ttf2]
    res["topk_canonical"] = [[[d, float(s)] for d, s in D.global_search(ad, q, K)] for q in QUERIES]
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()
    if idx is not None:
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


def expected_shard(world):
    texts, names = corpus()
    workers = []
    for r in range(world):
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
    assert res["canonical"] == [want["n_vocab"], want["dc"], want["ttf"]]

    def same(got, exp):
        assert [d for d, _ in got] == [d for d, _ in exp]
        assert [np.float32(s) for _, s in got] == [np.float32(s) for _, s in exp]

    for q, a, b, c, w in zip(QUERIES, res["topk"], res["batch"], res["topk_canonical"], want["topk"]):
        same(a, w)
        same(b, w)
        same(c, w)
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
    uni = [w.encode() for w in ("café", "naïve", "über", "façade", "señor", "ångström", "smörgåsbord",
                                 "crème", "brûlée", "jalapeño", "Ελλάδα", "москва", "日本語")]
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


class AttemptOracleAdapter(OracleShardAdapter):
    """Oracle adapter with a simulated hash-seed attempt: ``start`` is the
    attempt this shard's commit ended at; ``collide_at`` = attempts at which a
    recommit meets a collision (and moves on to the next)."""

    def __init__(self, texts, names, doc_base, start, collide_at=()):
        super().__init__(texts, names, doc_base)
        self.attempt = start
        self.collide_at = set(collide_at)
        self.recommits = []

    def hash_attempt(self):
        return self.attempt

    def recommit(self, attempt):
        self.recommits.append(attempt)
        while attempt in self.collide_at:
            attempt += 1
        self.attempt = attempt
        return attempt


def run_rank_seed(rank, world, port, kind, out_path):
    """kind "oracle": world 3, shard attempts (0, 1, 0); shard 2 collides again
    at attempt 1, so the ranks agree on 2 after two rounds.  kind "hip": the
    real engine, shard 1 (only) under TFIDF_TEST_WEAK_HASH (every pair of
    equal-length hashed keys collides: its commit moves to attempt 1)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    texts, names = seed_corpus()
    lo, hi = D.shard_range(len(texts), rank, world)
    idx = None
    if kind == "hip":
        from tfidf_amd.engine import ShardIndex
        torch.cuda.set_device(0)
        if rank == 1:
            os.environ["TFIDF_TEST_WEAK_HASH"] = "1"
        idx = ShardIndex(device=0)
        idx.add_documents(texts[lo:hi], names[lo:hi])
        idx.commit()
        os.environ.pop("TFIDF_TEST_WEAK_HASH", None)
        ad = D.HipShardAdapter(idx, torch.device("cuda", 0), doc_base=lo)
        before = ad.hash_attempt()
    else:
        ad = AttemptOracleAdapter(texts[lo:hi], names[lo:hi], lo, start=(0, 1, 0)[rank],
                                  collide_at=(1,) if rank == 2 else ())
        before = ad.hash_attempt()
    nv, dc, ttf = D.global_commit(ad, vocab_size=True)
    res = {"before": before, "after": ad.hash_attempt(), "n_vocab": nv, "dc": dc, "ttf": ttf,
           "recommits": getattr(ad, "recommits", None),
           "topk": [[[d, float(s)] for d, s in D.global_search(ad, q, K)] for q in _seed_queries()]}
    with open("%s.%d" % (out_path, rank), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()
    if idx is not None:
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
