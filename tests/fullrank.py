"""Rank body of the full-size multi-shard GPU tests (test_gpu_fullsize_multirank.py):
BASELINE cfg 3 (10 M docs over 8 shards, GLOBAL statistics, top-100 merge),
cfg 4 on 8 shards (10 k-query batch) and cfg 5 (50 M short docs, 5 M-term
vocabulary, over 8 shards).  The reference path this replaces is the fan-out
and merge of Leader.start (Leader.java:51-91) over the shards' Worker.searchIndex
(Worker.java:222-241), with one worker's (= global) statistics.

World 8 over gloo, every rank's ShardIndex on cuda:0 (RCCL needs one GPU per
rank; the 8-GPU RCCL run is the driver's).  Rank r generates documents
[r N/8, (r+1) N/8) of the global synthetic corpus in HBM (DeviceCorpus,
doc_base) and indexes them; the ranks exchange statistics with the production
code (the library's tfidf_dist_global_commit, through distributed.DistShard
over a callback communicator on the gloo group) and answer queries with it
(tfidf_dist_search / tfidf_dist_search_batch).  Checks, none of which use an oracle
index of the whole corpus (it would not finish in a test):

* every shard's df of its WHOLE vocabulary = an independent torch count of its
  own bytes (test_gpu_fullsize.independent_df: word spans and byte keys with
  plain tensor ops, none of the engine's kernels); the GLOBAL df in force for
  every term of every shard = the sum over ranks of those independent counts;
  the global vocabulary size = the number of distinct terms over all shards;
* docCount = N and sumTotalTermFreq = sum of the generator's document lengths;
* global_search(k=100): (score desc, doc asc) order; every hit's score
  recomputed bit-exactly by the rank that holds the document, with the
  oracle's Lucene arithmetic (oracle.idf / avgdl / norm_cache / bm25) from the
  global statistics and the hit's TF row; the merged list = the top-100 of the
  union of the shards' own top-100 lists; one-term all-hits counts = global df;
* completeness: the merged top-100 of multi-term queries = the top-100 of
  every document of the node that holds a query term, each scored from the
  corpus bytes alone (span keys -> tf, generator lengths -> norms) with the
  independent global statistics (test_gpu_fullsize.independent_topk);
* the 10 k-query batch merged over the shards = per-query searches.

Every rank records failed checks instead of raising (a raising rank would
leave the others in a collective); rank files are asserted by the parent.
"""
import datetime
import json
import os

import numpy as np
import torch
import torch.distributed as dist

from oracle import oracle as O
from tfidf_amd import distributed as D
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

from test_gpu_fullsize import f32bits, independent_df, independent_topk, span_keys, term_lo

K1, B = 1.2, 0.75

CFGS = {
    # BASELINE configs[2] / [3]: 10 M docs x U[400, 600] tokens, V = 100 k, 8 shards
    "cfg3": dict(n_total=10_000_000, V=100_000, len_min=400, len_max=600, cap=18,
                 queries=lambda: synth.queries(24),
                 batch=lambda: synth.queries(10_000)),
    # BASELINE configs[4]: 50 M docs x U[48, 80] tokens, V = 5 M, 8 shards
    "cfg5": dict(n_total=50_000_000, V=5_000_000, len_min=48, len_max=80, cap=23,
                 queries=lambda: synth.queries(16, lo=100, hi=20_000) +
                 synth.queries(8, lo=100_000, hi=4_000_000, seed=9),
                 batch=lambda: synth.queries(2_000, lo=100, hi=200_000)),
}
TOPK = 100


def doc_lengths_range(base, n, len_min, len_max, seed=synth.SEED):
    """T_d of documents base .. base + n - 1 (the generator's definition)."""
    s2 = synth._mix64(np.uint64(seed))
    d = np.arange(base, base + n, dtype=np.uint64)
    h = synth._mix64(s2 ^ ((d << np.uint64(20)) | np.uint64(0xFFFFF)))
    return len_min + (h % np.uint64(len_max - len_min + 1)).astype(np.int64)


def _gather_var(a):
    """1-D int64 numpy arrays of every rank, concatenated in rank order (gloo)."""
    n = torch.tensor([len(a)], dtype=torch.int64)
    ns = [torch.zeros(1, dtype=torch.int64) for _ in range(dist.get_world_size())]
    dist.all_gather(ns, n)
    m = max(int(x.item()) for x in ns)
    pad = torch.zeros(max(m, 1), dtype=torch.int64)
    pad[:len(a)] = torch.from_numpy(np.ascontiguousarray(a, np.int64))
    parts = [torch.zeros(max(m, 1), dtype=torch.int64) for _ in ns]
    dist.all_gather(parts, pad)
    return np.concatenate([p[:int(k.item())].numpy() for p, k in zip(parts, ns)])


def _gather_obj(x, world):
    out = [None] * world
    dist.all_gather_object(out, x)
    return out


def run(rank, world, port, cfg, out_path, concurrent_counts=2):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=900))
    torch.cuda.set_device(0)
    c = CFGS[cfg]
    n_total = c["n_total"]
    n = n_total // world
    base = rank * n
    errors = []
    info = {"rank": rank, "docs": n}

    def check(cond, msg):
        if not cond:
            errors.append(msg)

    def progress(what):
        if rank == 0:
            print("[%s rank 0] %s" % (cfg, what), flush=True)

    dc = synth.DeviceCorpus(n, V=c["V"], len_min=c["len_min"], len_max=c["len_max"], doc_base=base)
    g = ShardIndex(vocab_capacity_log2=c["cap"])
    g.add_documents_device(dc.d_text, dc.d_offsets, dc.n_docs, dc.total_bytes)
    g.commit()
    st = g.stats()
    info.update(nnz=st["nnz"], terms=st["num_terms"], term_major=st["term_major"])
    comm = D.Comm.from_group(transport="callback")
    ad = D.DistShard(g, comm, doc_base=base)
    n_vocab, gdc, gttf = ad.global_commit(vocab_size=True)
    torch.cuda.synchronize()
    progress("built and exchanged: %d docs, %d terms locally, %d globally" % (n, st["num_terms"], n_vocab))

    # ---- statistics -------------------------------------------------------
    lens = doc_lengths_range(base, n, c["len_min"], c["len_max"])
    check(st["num_docs"] == n and st["doc_count"] == n, "local doc count")
    check(st["sum_ttf"] == int(lens.sum()), "local sumTTF != generator")
    tot = torch.tensor([int(lens.sum())], dtype=torch.int64)
    dist.all_reduce(tot)
    check(gdc == n_total, "global docCount %d != %d" % (gdc, n_total))
    check(gttf == int(tot.item()), "global sumTTF %d != generator %d" % (gttf, int(tot.item())))
    # independent per-shard counts, a few ranks at a time (GPU memory)
    ind = None
    for turn in range(0, world, concurrent_counts):
        if turn <= rank < turn + concurrent_counts:
            ind = independent_df(dc, n)
        dist.barrier()
    keys, dl, de = g.vocab_export()
    check(bool((keys[:, 1] == np.uint64(1 << 63)).all()), "a term over 8 bytes in the synthetic vocabulary")
    lo = keys[:, 0].astype(np.int64)
    check(dict(zip(lo.tolist(), dl.tolist())) == ind, "local df != independent count of the shard")
    ind_lo = np.fromiter(ind.keys(), np.int64, len(ind))
    ind_df = np.fromiter(ind.values(), np.int64, len(ind))
    del ind
    glo = _gather_var(ind_lo)
    gdf = _gather_var(ind_df)
    uk, inv = np.unique(glo, return_inverse=True)
    gsum = np.bincount(inv, weights=gdf).astype(np.int64)
    del glo, gdf, inv
    check(n_vocab == len(uk), "global vocabulary %d != %d distinct terms over the shards" % (n_vocab, len(uk)))
    pos = np.searchsorted(uk, lo)
    check(bool((uk[pos] == lo).all()), "local term missing from the gathered vocabulary")
    bad = np.nonzero(gsum[pos] != de.astype(np.int64))[0]
    check(bad.size == 0, "%d terms' GLOBAL df != sum of independent shard counts" % bad.size)
    info["global_vocab"] = int(len(uk))
    progress("statistics checked")

    # ---- completeness: the merged top-100 = the top-100 of EVERY document of
    # the node holding a query term, scored from the corpus bytes alone with
    # the independent GLOBAL statistics (each rank scores its own documents;
    # the candidates meet on the host) — no engine kernel involved
    def gdf_of(term):
        kk = term_lo(term)
        i = int(np.searchsorted(uk, kk))
        return int(gsum[i]) if i < len(uk) and uk[i] == kk else 0

    qs_c = c["queries"]()[:8]
    cand = None
    for turn in range(0, world, concurrent_counts):
        if turn <= rank < turn + concurrent_counts:
            key, dk = span_keys(dc, n)
            cand = independent_topk(key, dk, n, base, qs_c, TOPK, gdf_of, n_total, int(tot.item()), lens)
            del key, dk
            torch.cuda.empty_cache()
        dist.barrier()
    allc = _gather_obj(cand, world)
    for qi, q in enumerate(qs_c):
        union = sorted([x for part in allc for x in part[qi]], key=lambda x: (-x[1], x[0]))[:TOPK]
        hits = ad.search(q, TOPK)
        check([d for d, _ in hits] == [d for d, _ in union], "query %r: merged top-%d misses documents" % (q, TOPK))
        check([f32bits(x) for _, x in hits] == [f32bits(x) for _, x in union],
              "query %r: merged top-%d scores != independent" % (q, TOPK))
    del allc, cand
    progress("completeness checked")

    # ---- top-100 over the shards -----------------------------------------
    cache = O.norm_cache(K1, B, O.avgdl(gttf, gdc))
    gdf_of = dict(zip(lo.tolist(), de.tolist()))

    def df_global(term):
        k = int.from_bytes(term.ljust(8, b"\0"), "little")
        return gdf_of.get(k, 0)

    def expected(q_terms, d_local):
        row = g.doc_terms(d_local)
        _, nrm = g.doc_len(d_local)
        acc = 0.0
        for t in q_terms:
            if t in row:
                acc += float(O.bm25(O.idf(df_global(t), gdc), row[t], float(cache[nrm])))
        return f32bits(float(np.float32(acc)))

    qs = c["queries"]()
    n_checked = 0
    for q in qs:
        hits = ad.search(q, TOPK)
        check(len(hits) == TOPK, "query %r: %d hits" % (q, len(hits)))
        ks = [(-s, d) for d, s in hits]
        check(ks == sorted(ks), "query %r: not (score desc, doc asc)" % q)
        terms = q.split(b" ")
        for d, s in hits:
            if base <= d < base + n:
                n_checked += 1
                check(f32bits(s) == expected(terms, d - base), "query %r doc %d: score bits" % (q, d))
        # the merge: top-100 of the union of every shard's own top-100 (host lists)
        mine = [(d + base, s) for d, s in g.search(q, TOPK)]
        union = [x for part in _gather_obj(mine, world) for x in part]
        union.sort(key=lambda x: (-x[1], x[0]))
        check(hits == union[:TOPK], "query %r: merged top-%d != top of the shards' lists" % (q, TOPK))
    info["scores_checked"] = n_checked
    progress("top-%d checked" % TOPK)
    for q in qs[:3]:                                     # one term, every hit: exactly the global df
        t = q.split(b" ")[0]
        allh = ad.search(t, 0)
        check(len(allh) == df_global(t) or df_global(t) == 0, "all hits of %r: %d" % (t, len(allh)))
        ks = [(-s, d) for d, s in allh]
        check(ks == sorted(ks), "all hits of %r: order" % t)

    # ---- cfg 4 on the shards: the batch merged once = per-query searches ---
    bq = c["batch"]()
    bd, bs, bc = ad.search_batch(bq, 10)
    step = max(1, len(bq) // 150)
    for i in range(0, len(bq), step):
        one = ad.search(bq[i], 10)
        got = list(zip(bd[i, :bc[i]].tolist(), bs[i, :bc[i]].tolist()))
        check(got == one, "batch query %d != global_search" % i)
    info["batch_queries"] = len(bq)
    progress("batch checked")

    with open("%s.%d" % (out_path, rank), "w") as f:
        json.dump({"errors": errors, "info": info}, f)
    dist.barrier()
    comm.close()
    dist.destroy_process_group()
    g.close()
    dc.free()


def check_ranks(out_path, world):
    res = [json.load(open("%s.%d" % (out_path, r))) for r in range(world)]
    errs = [(r, e) for r, x in enumerate(res) for e in x["errors"]]
    assert not errs, errs[:20]
    return [x["info"] for x in res]
