"""World-size-2 (and 3) CPU rehearsal of the multi-GPU orchestration in
tfidf_amd/distributed.py over the gloo backend.  The per-rank engine is the
CPU oracle behind the same adapter interface HipShardAdapter implements; the
orchestration code under test (vocabulary all-gather, canonical DF
all-reduce, per-rank top-k all-gather + merge) is the production code.

GLOBAL mode over G shards must equal the single-index (1-worker) result.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O
from tfidf_amd import distributed as D
from tfidf_amd import synth
from tfidf_amd.engine import term_key

N_DOCS = 1200


class OracleShardAdapter:
    device = torch.device("cpu")

    def __init__(self, texts, doc_base):
        self.o = O.OracleIndex()
        for i, t in enumerate(texts):
            self.o.add_doc(str(doc_base + i).encode(), t)
        self.o.commit()
        self.doc_base = doc_base

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

    # term-ownership exchange (distributed.global_commit)
    @staticmethod
    def _owner(lo, hi, G):
        return ((lo * 0x9E3779B97F4A7C15 ^ hi) & 0xFFFFFFFFFFFFFFFF) % G

    def vocab_partition(self, n_ranks):
        groups = [[] for _ in range(n_ranks)]
        self.sent_terms = []
        by_owner = [[] for _ in range(n_ranks)]
        for t, df in sorted(self.o.vocab().items()):
            lo, hi = term_key(t)
            r = self._owner(lo, hi, n_ranks)
            groups[r].append((lo, hi, df))
            by_owner[r].append(t)
        for r in range(n_ranks):
            self.sent_terms += by_owner[r]
        rows = [x for g in groups for x in g]
        rec = np.array(rows, np.uint64).reshape(-1, 3).view(np.int64)
        return torch.from_numpy(rec.copy()), [len(g) for g in groups]

    def vocab_reduce(self, records):
        r = records.numpy().view(np.uint64)
        tot = {}
        for lo, hi, df in r.tolist():
            tot[(lo, hi)] = tot.get((lo, hi), 0) + df
        ans = np.array([tot[(lo, hi)] for lo, hi, _ in r.tolist()], np.int32)
        return torch.from_numpy(ans), len(tot)

    def import_global_df(self, gdf, doc_count, sum_ttf):
        g = gdf.numpy().tolist()
        self.o.set_global_stats(doc_count, sum_ttf, {t: int(d) for t, d in zip(self.sent_terms, g)})

    def import_global(self, dfc, doc_count, sum_ttf):
        dfc = dfc.numpy()
        df_by_term = {t: int(dfc[self.canon_index[key]]) for key, t in self.terms.items()}
        self.o.set_global_stats(doc_count, sum_ttf, df_by_term)

    def search_topk(self, q, k):
        hits = self.o.search(q, k)
        return np.array([d for d, _ in hits], np.uint32), np.array([s for _, s in hits], np.float32)

    def search_batch(self, queries, k):
        docs = np.zeros((len(queries), k), np.uint32)
        scores = np.zeros((len(queries), k), np.float32)
        counts = np.zeros(len(queries), np.uint32)
        for i, q in enumerate(queries):
            d, s = self.search_topk(q, k)
            docs[i, :len(d)], scores[i, :len(s)], counts[i] = d, s, len(d)
        return docs, scores, counts


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, queries, k, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    texts = synth.corpus(N_DOCS, V=6000, len_min=20, len_max=150)
    lo, hi = D.shard_range(N_DOCS, rank, world)
    ad = OracleShardAdapter(texts[lo:hi], lo)
    n_canon, dc, ttf = D.global_commit(ad)
    results = [D.global_search(ad, q, k) for q in queries]
    # the canonical (all-gather + sorted union) form must agree
    n2, dc2, ttf2 = D.global_commit_canonical(ad)
    assert (n2, dc2, ttf2) == (n_canon, dc, ttf)
    assert [D.global_search(ad, q, k) for q in queries] == results
    D.global_commit(ad)
    bd, bs, bc = D.global_search_batch(ad, queries, k)
    batch = [[[int(bd[i, j]), float(bs[i, j])] for j in range(int(bc[i]))] for i in range(len(queries))]
    if rank == 0:
        import json
        with open(out_path, "w") as f:
            json.dump({"n_canon": n_canon, "dc": dc, "ttf": ttf, "batch": batch,
                       "results": [[[d, float(s)] for d, s in r] for r in results]}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_global_mode_equals_single_index(tmp_path, world):
    queries = synth.queries(12, lo=1, hi=1500) + [b"aaaa", b"aaab aaac"]
    k = 25
    out = str(tmp_path / "r.json")
    mp.spawn(_worker, args=(world, _free_port(), queries, k, out), nprocs=world, join=True)
    import json
    res = json.load(open(out))
    texts = synth.corpus(N_DOCS, V=6000, len_min=20, len_max=150)
    o = O.OracleIndex()
    for i, t in enumerate(texts):
        o.add_doc(str(i).encode(), t)
    o.commit()
    assert res["dc"] == o.doc_count and res["ttf"] == o.sum_ttf
    assert res["n_canon"] == o.num_terms
    for q, got, gotb in zip(queries, res["results"], res["batch"]):
        want = o.search(q, k)
        assert [d for d, _ in got] == [d for d, _ in want]
        assert [np.float32(s) for _, s in got] == [np.float32(s) for _, s in want]
        assert [d for d, _ in gotb] == [d for d, _ in want]
        assert [np.float32(s) for _, s in gotb] == [np.float32(s) for _, s in want]
