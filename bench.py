#!/usr/bin/env python3
"""bench.py — docs indexed/sec (+ queries scored/sec) on MI355X.

Workload (BASELINE.json configs[1], "cfg 2"): synthetic Zipf(s=1) corpus,
1M documents x U[400,600] tokens, 100k-term vocabulary, generated directly in
HBM (synthetic data: no network for real corpora).  One step = one full index
build (tfidf_commit: tokenise + per-doc TF rows + DF + inverted postings) of
the HBM-resident corpus on every rank; with N > 1 GPUs each rank owns its own
1M-doc shard (weak scaling, BASELINE cfg 3 layout) and a step also runs the
GLOBAL-statistics exchange (vocabulary all-gather + DF all-reduce over RCCL).
Query throughput is measured after the timed region: cfg-2 single 3-term
queries (top-10 and all-hits) and cfg-4 batched 10k queries (top-10).

Launch: python bench.py [--gpus N --steps K --warmup W].  N > 1 runs one
process per GPU (RCCL): under torch.distributed.run (WORLD_SIZE must equal N),
or, started without a launcher, bench.py starts torch.distributed.run with N
ranks itself as a child process before touching the GPU and exits with its
return code (rank 0's JSON line reaches the same stdout).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tf-idf-distributed-system_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec



def default_cap(vocab):
    """Dictionary slots (log2) for a vocabulary: load <= 0.25 while the
    block-major inversion applies (<= 2^21 slots; its count table is sized by
    the vocabulary, so a sparser probe table costs only the table itself and
    resolves nearly every tokenizer lookup in its first probe round), else
    the smallest power of two >= 1.6 x vocab (term-major, cfg 5)."""
    cap = 18
    while (1 << cap) < 4 * vocab and cap < 21:
        cap += 1
    if (1 << cap) < 4 * vocab:
        cap = 18
        while (1 << cap) < 1.6 * vocab:
            cap += 1
    return cap

def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--docs", type=int, default=1_000_000, help="documents per GPU")
    ap.add_argument("--vocab", type=int, default=100_000)
    ap.add_argument("--len-min", type=int, default=400)
    ap.add_argument("--len-max", type=int, default=600)
    ap.add_argument("--queries", type=int, default=200, help="single-query timing repetitions")
    ap.add_argument("--batch-queries", type=int, default=10_000)
    ap.add_argument("--cpu-sample", type=int, default=25_000, help="docs in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--no-queries", action="store_true")
    ap.add_argument("--cap-log2", type=int, default=0,
                    help="dictionary slots 2^x (0 = default_cap(vocab))")
    ap.add_argument("--inversion", choices=("auto", "block", "term"), default="auto")
    ap.add_argument("--unicode-every", type=int, default=0,
                    help="one non-ASCII word per this many bytes of every document (book-like text)")
    ap.add_argument("--prose", type=float, default=0.0,
                    help="prose typography (curly quotes, apostrophes, dashes, accented and capital letters) "
                         "at this multiple of synth.DeviceCorpus.PROSE's rates (0 = plain synthetic words)")
    ap.add_argument("--unicode-frac", type=float, default=0.0,
                    help="fraction of documents made non-ASCII (Unicode tokenizer path); 0 = the cfg-2 corpus")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false",
                    help="skip the PCIe-inclusive (host corpus -> HBM -> index) measurement")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "r06", "traffic.json"),
                    help="per-kernel HBM bytes from tools/prof_round.sh (rocprofv3 PMC passes of this workload)")
    return ap.parse_args()


def launcher_cmd(n_gpus, argv, port=None):
    """torch.distributed.run command that runs this script with n_gpus ranks."""
    if port is None:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n_gpus,
            "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)


def launch_or_check(args, argv):
    """None to run here; else the exit code.  --gpus N > 1 without a launcher
    (WORLD_SIZE unset): run N ranks under torch.distributed.run as a child
    (nothing here has touched the GPU yet); under a launcher WORLD_SIZE must be N."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus > 1:
            return subprocess.call(launcher_cmd(args.gpus, argv))
        return None
    if int(ws) != args.gpus:
        print("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks" % (args.gpus, ws), file=sys.stderr)
        return 2
    return None


def cpu_threads():
    """Threads for the all-cores CPU baseline: the CPUs this process may run
    on, capped by the GPU box's per-GPU CPU share (the pool allots 16 CPUs per
    GPU and exports OMP_NUM_THREADS=16; os.cpu_count() / the affinity mask
    show the whole 8-GPU machine).  -> (threads, reason)."""
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if share and share < usable:
        return share, ("OMP_NUM_THREADS=%d: the box's CPU share for this one GPU (%d CPUs usable are the whole "
                       "machine's, shared with the other GPUs' jobs)" % (share, usable))
    return usable, "all usable CPUs (sched_getaffinity)"


def cpu_baseline(corpus, args, n_docs):
    """Reference-semantics CPU restatement (oracle/, C) on the same corpus:
    docs indexed/sec by C threads with no Python in the timed region
    (orc_bulk_build): 1 thread over the first n_docs, then T threads each
    indexing its own n_docs-doc share (the reference's N-worker layout, one
    IndexWriter per worker) and the scaling curve 1, 2, 4, ... T; top-10 and
    all-hits + materialised (name, score) JSON query rates on an n_docs index."""
    from oracle import oracle as O
    from tfidf_amd import synth
    T, why = cpu_threads()
    T = max(1, min(T, corpus.n_docs // n_docs))
    n = min(n_docs, corpus.n_docs)
    text, offs = corpus.to_host(n * T)
    # single thread: the first n documents
    t_idx, ttf1 = O.bulk_build(text[:int(offs[n])], offs[:n + 1], 1)
    # scaling curve: t threads over t * n documents (each thread's index as large as the single one's)
    curve = {}
    t = 2
    while t <= T:
        sec, _ = O.bulk_build(text[:int(offs[t * n])], offs[:t * n + 1], t)
        curve[t] = t * n / sec
        t *= 2
    if T > 1 and T not in curve:
        sec, _ = O.bulk_build(text, offs, T)
        curve[T] = T * n / sec
    raw = text[:int(offs[n])].tobytes()
    del text
    o = O.OracleIndex()
    for i in range(n):
        o.add_doc(str(i).encode(), raw[int(offs[i]):int(offs[i + 1])])
    o.commit()
    qs = synth.queries(50)
    t0 = time.perf_counter()
    for q in qs:
        o.search(q, 10)
    t_q = time.perf_counter() - t0
    t0 = time.perf_counter()
    for q in qs[:10]:
        hits = o.search(q, 0)
        json.dumps([{"document": {"name": o.doc_key(d).decode()}, "score": float(sc)} for d, sc in hits])
    t_all = time.perf_counter() - t0
    o.close()
    # the GPU engine on the SAME sample and queries (comparable query rates)
    from tfidf_amd.engine import ShardIndex
    g = ShardIndex()
    g.add_documents([raw[int(offs[i]):int(offs[i + 1])] for i in range(n)], [str(i).encode() for i in range(n)])
    g.commit()
    g.search(qs[0], 10)
    t0 = time.perf_counter()
    for q in qs:
        g.search(q, 10)
    g_q = time.perf_counter() - t0
    blob, koffs = g.doc_keys()                   # every name once (the index's stored field)
    blob = bytes(blob)
    t0 = time.perf_counter()
    for q in qs[:10]:
        docs, scs = g.search_all_arrays(q)
        ko = koffs[docs.astype(np.int64)]
        ke = koffs[docs.astype(np.int64) + 1]
        json.dumps([{"document": {"name": blob[a:b].decode()}, "score": float(sc)}
                    for a, b, sc in zip(ko.tolist(), ke.tolist(), scs.tolist())])
    g_all = time.perf_counter() - t0
    g.close()
    single = n / t_idx
    out = {"value": single, "unit": "docs/s", "cores": 1, "kind": "port",
           "sample": "first %d docs (%.1f MB) of the same synthetic corpus, oracle/ C restatement of "
                     "Lucene 9.8 analysis+inversion+stats, 1 C thread (no Python in the timed region); "
                     "no JDK/Lucene in the image" % (n, float(offs[n]) / 1e6),
           "seconds": t_idx, "sum_ttf": ttf1, "queries_per_sec_top10": len(qs) / t_q,
           "queries_per_sec_all_hits_materialised": 10 / t_all,
           "queries_sample": "cfg-2 queries over the %d-doc sample (all hits: + doc key lookup + JSON, "
                             "as Worker.searchIndex)" % n,
           "gpu_same_sample": {"queries_per_sec_top10": len(qs) / g_q,
                               "queries_per_sec_all_hits_materialised": 10 / g_all,
                               "note": "libtfidf on the same sample and queries, through the C ABI from Python"},
           "host_cpus": os.cpu_count(),
           "host_cpus_usable": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}
    if T > 1:
        out["all_cores"] = {"value": curve[T], "unit": "docs/s", "threads": T, "threads_reason": why,
                            "seconds": T * n / curve[T], "scaling_efficiency": curve[T] / (T * single),
                            "curve_docs_per_s": {str(k): v for k, v in sorted(curve.items())},
                            "sample": "%d C threads (orc_bulk_build), each indexing its own %d-doc share of the "
                                      "same corpus into its own index" % (T, n)}
    return out


def measured_copy_GBs(dev, nbytes=1 << 30, reps=5):
    """Device-to-device copy bandwidth (read + write bytes / time): the
    achievable-HBM reference the roofline is also quoted against."""
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2 * nbytes / (ms * 1e-3) / 1e9


def bench_node(args):
    """TFIDF_BENCH_NODE=1: process model (1) of include/tfidf.h — ONE process
    owns --gpus N devices through tfidf_node (device mask (1 << N) - 1, RCCL
    communicator from ncclCommInitAll, one worker thread per shard): the ABI a
    Java host binds.  Each shard's 1M-doc corpus is
    generated on its own GPU; a timed step = tfidf_node_commit (every shard's
    build in parallel + the GLOBAL statistics exchange); then node-level batched
    and single GLOBAL queries.  Prints one JSON line (not the driver's line)."""
    import ctypes as C
    import torch
    from tfidf_amd import _lib as L
    from tfidf_amd import synth
    from tfidf_amd import distributed as D
    G = args.gpus
    torch.cuda.set_device(0)
    cap = args.cap_log2 or default_cap(args.vocab)
    node = D.Node(devices=list(range(G)), stats_mode=L.STATS_GLOBAL, vocab_capacity_log2=cap)
    lib = L.load()
    corpora = []
    for g in range(G):
        c = synth.DeviceCorpus(args.docs, V=args.vocab, len_min=args.len_min, len_max=args.len_max,
                               doc_base=g * args.docs, device=g)
        L.check(lib.tfidf_add_docs_device(node.shard(g), C.c_void_p(c.d_text), C.c_void_p(c.d_offsets), args.docs,
                                          c.total_bytes))
        corpora.append(c)
    for _ in range(args.warmup):
        node.commit()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        node.commit()
    elapsed = time.perf_counter() - t0
    st = node.stats()
    per_shard = []
    for g in range(G):
        t = L.CommitTiming()
        L.check(lib.tfidf_get_commit_timing(node.shard(g), C.byref(t)))
        per_shard.append(t.ms_total)
    out = {
        "metric": "docs indexed/sec + queries scored/sec (node) at 1/2/4/8 GPUs; % HBM roofline",
        "value": st["num_docs"] * args.steps / elapsed, "unit": "docs/s", "n_gpus": G, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "u8/u32 (integer inversion), f32 BM25 with f64 accumulation",
        "data": "synthetic (Zipf s=1.0 corpus generated in HBM by tfidf_synth_corpus, seed 20251015)",
        "config": {"workload": "cfg2 per shard: %d docs/GPU x U[%d,%d] tokens, V=%d; tfidf_node_commit = every "
                               "shard's build + GLOBAL stats exchange" % (args.docs, args.len_min, args.len_max,
                                                                          args.vocab),
                   "process_model": "node: one process, tfidf_node over device mask 0x%x (include/tfidf.h (1))"
                                    % ((1 << G) - 1),
                   "transport": {1: "rccl", 2: "inproc"}.get(st["transport"], st["transport"]),
                   "docs": st["num_docs"], "global_vocab": st["num_terms"], "parallelism": "dp%d" % G},
        "shard_build_device_ms": per_shard,
    }
    if not args.no_queries:
        bq = synth.queries(args.batch_queries)
        node.search_batch(bq[:100], 10)
        for k in (10, 100):
            t0 = time.perf_counter()
            node.search_batch(bq, k)
            out["batch%dk_top%d_qps" % (len(bq) // 1000, k)] = len(bq) / (time.perf_counter() - t0)
        qs = synth.queries(max(args.queries, 1))
        node.search(qs[0], 10)
        lat = []
        for q in qs:
            t1 = time.perf_counter()
            node.search(q, 10)
            lat.append(time.perf_counter() - t1)
        out["single_top10_p50_ms"] = float(np.percentile(lat, 50)) * 1e3
        out["single_top10_qps"] = len(qs) / sum(lat)
    node.close()
    for c in corpora:
        c.free()
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if os.environ.get("TFIDF_BENCH_NODE") == "1":
        return bench_node(args)
    rc = launch_or_check(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # multi-GPU code path (process group, GLOBAL statistics exchange) even at
    # one rank: TFIDF_BENCH_DIST=1 rehearses the RCCL collectives on a 1-GPU box
    dist_on = world > 1 or os.environ.get("TFIDF_BENCH_DIST") == "1"
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # one process per GPU; the modulo only matters for a rehearsal with more
    # ranks than GPUs (TFIDF_BENCH_BACKEND=gloo on a 1-GPU box)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist_on:
        # the process group only bootstraps (RCCL unique id, barriers, the
        # max-over-ranks time); the data-path collectives are the library's
        # own RCCL communicator (over xGMI), or with TFIDF_BENCH_BACKEND=gloo
        # (ranks sharing a GPU in a rehearsal) the group's collectives as callbacks
        dist.init_process_group("gloo")

    def barrier():
        if dist_on:
            dist.barrier()

    from tfidf_amd import STATS_GLOBAL, synth
    from tfidf_amd import distributed as D
    from tfidf_amd.engine import ShardIndex

    n_docs = args.docs
    doc_base = rank * n_docs
    corpus = synth.DeviceCorpus(n_docs, V=args.vocab, len_min=args.len_min, len_max=args.len_max,
                                doc_base=doc_base, device=local)
    n_unicode = corpus.inject_unicode(args.unicode_frac) + corpus.inject_unicode_every(args.unicode_every)
    n_prose = corpus.inject_prose(args.prose)
    cap = args.cap_log2 or default_cap(args.vocab)
    inv = {"auto": 0, "block": 1, "term": 2}[args.inversion]
    idx = ShardIndex(device=local, vocab_capacity_log2=cap, inversion=inv,
                     stats_mode=STATS_GLOBAL if dist_on else 0)
    idx.add_documents_device(corpus.d_text, corpus.d_offsets, n_docs, corpus.total_bytes)
    adapter = None
    if dist_on:
        transport = "callback" if os.environ.get("TFIDF_BENCH_BACKEND", "rccl") == "gloo" else "rccl"
        comm = D.Comm.from_group(device=local, transport=transport)
        adapter = D.DistShard(idx, comm, doc_base=doc_base)

    exch = [0.0]

    def step():
        idx.commit()                     # returns with the build complete (its stream synced)
        if dist_on:
            # GLOBAL statistics: term-ownership all-to-alls + stats all-gather
            # (libtfidf tfidf_dist_global_commit; timed on the host: the commit
            # is already complete here)
            t1 = time.perf_counter()
            adapter.global_commit()
            torch.cuda.synchronize()
            exch[0] += time.perf_counter() - t1

    for _ in range(args.warmup):
        step()
    exch[0] = 0.0
    phases = {k: 0.0 for k in ("ms_tokenize", "ms_long", "ms_df", "ms_blockscan", "ms_colscan", "ms_scatter",
                                "ms_total")}
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        t = idx.commit_timing()
        for k in phases:
            phases[k] += t[k]
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    for k in phases:
        phases[k] /= args.steps
    st = idx.stats()
    timing = idx.commit_timing()
    text_bytes, nnz, N = st["text_bytes"], st["nnz"], st["num_docs"]

    # ---- roofline of the dominant kernel (algorithmic bytes) ----
    copy_gbs = measured_copy_GBs(dev)
    C_slots = 1 << cap
    n_blocks = (N + 8191) // 8192
    if st["term_major"]:
        n_blocks = 0        # no per-block count table: the sort-based inversion reads CSR, writes postings
    alg = {
        # text read once + CSR (slot u32 + tf u32) written once + row metadata (SURVEY: 9 B/doc)
        "ms_tokenize": text_bytes + 8 * nnz + 9 * N,
        # long-document path (book-sized documents): the same formula over the documents it takes
        "ms_long": text_bytes + 8 * nnz + 9 * N,
        # slot column read + per-block DF partials written
        "ms_df": 4 * nnz + 4 * n_blocks * C_slots,
        # partials read + offsets written
        "ms_blockscan": 12 * n_blocks * C_slots,
        # CSR (slot + tf) read + packed postings written
        "ms_scatter": 16 * nnz + 4 * n_blocks * C_slots,
    }
    dom = max(alg, key=lambda k: phases[k])
    dom_ms = phases[dom]
    achieved = alg[dom] / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    phase_gbs = {k: (alg[k] / (phases[k] * 1e-3) / 1e9 if phases[k] > 0 else None) for k in alg}
    b_index = text_bytes + 8 * nnz + 9 * N + 4 * args.vocab * world
    # measured HBM traffic of the dominant kernel: a separate rocprofv3 PMC pass
    # over the same workload (counters cannot be read from inside this run)
    traffic, traffic_src = None, None
    kname = {"ms_tokenize": "k_tokenize_wave", "ms_long": "k_tokenize_long", "ms_df": "k_df_partial",
             "ms_blockscan": "k_row_scan", "ms_scatter": "k_scatter"}[dom]
    try:
        tj = json.load(open(args.traffic_json))
        w = tj.get("workload") or {}
        if (w.get("docs_per_gpu"), w.get("text_bytes_per_gpu"), w.get("nnz_per_gpu")) == (N, text_bytes, nnz):
            # rocprof names carry template arguments (k_tokenize_wave<false>); a
            # phase of several kernels (k_scatter_part + k_scatter_sort) sums them
            hits = [v["hbm_bytes_corrected"] for n, v in tj["kernels"].items()
                    if n.split("<")[0] == kname or n.startswith(kname + "_")]
            traffic = sum(hits) if hits else None
            traffic_src = os.path.relpath(args.traffic_json, REPO) + " (" + tj["note"] + ")"
    except (OSError, KeyError, ValueError, TypeError):
        pass
    result = {
        "metric": "docs indexed/sec + queries scored/sec (node) at 1/2/4/8 GPUs; % HBM roofline",
        "value": world * N * args.steps / elapsed,
        "unit": "docs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/u32 (integer inversion), f32 BM25 with f64 accumulation",
        "data": "synthetic (Zipf s=1.0 corpus generated in HBM by tfidf_synth_corpus, seed 20251015)",
        "config": {"workload": "%s: %d docs/GPU x U[%d,%d] tokens, V=%d, full index build per step%s" % (
            "cfg2" if (args.vocab, args.len_min, args.len_max) == (100_000, 400, 600) else
            "cfg5-shape" if args.vocab >= 1_000_000 else "custom",
            N, args.len_min, args.len_max, args.vocab,
            "; GLOBAL stats exchange (term-ownership all-to-all of (term, df) records + stats all-reduce, RCCL)" if dist_on else ""),
            "docs_per_gpu": N, "text_bytes_per_gpu": text_bytes, "nnz_per_gpu": nnz,
            "vocab_terms": st["num_terms"], "dict_slots_log2": cap, "inversion": "term-major" if st["term_major"] else "block-major",
            "parallelism": "dp%d (document shards)" % world},
        "roofline": {"bound": "hbm", "kernel": dom.replace("ms_", ""), "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "measured_copy_GBs": copy_gbs, "frac_of_measured_copy": achieved / copy_gbs,
                     "traffic_source": traffic_src, "alg_bytes_per_launch": alg[dom], "avg_launch_ms": dom_ms},
        "phases_ms": phases,
        "phases_alg_GBs": phase_gbs,
        "index_build_alg_bytes": b_index,
        "index_build_GBs_end_to_end": b_index / (elapsed / args.steps) / 1e9,
        "global_exchange_ms_per_step": exch[0] * 1e3 / args.steps if dist_on else None,
        "global_exchange_frac_of_step": (exch[0] / elapsed) if dist_on else None,
        "long_docs": st["long_docs"],
        "long_chunked": st["long_chunked"],
        "hash_rebuilds": st["hash_rebuilds"],
        "engine_unicode_docs": st["unicode_docs"],
        "engine_unicode_wave_docs": st["unicode_wave_docs"],
        "unicode_docs": n_unicode,
        "prose_words": n_prose,
        "tokenizer_docs_per_window": st["pack_docs"],
        "pack_retried_docs": st["pack_retried"],
    }

    # ---- queries (outside the timed region) ----
    if not args.no_queries and not dist_on:
        from tfidf_amd.engine import analyze
        qs = synth.queries(max(args.queries, 1))
        # algorithmic bytes: 9 B per posting read (doc u32 + tf u32 + norm u8)
        df_cache = {}

        def post_bytes(q):
            tot = 0
            for t in set(analyze(q)):
                if t not in df_cache:
                    df_cache[t] = idx.df(t)[0]
                tot += 9 * df_cache[t]
            return tot

        idx.search(qs[0], 10)
        # latency / rate with query timing off (the serving configuration: the
        # HIP event records cost ~17 us per query), device time in a second pass
        idx.set_query_timing(False)
        lat = []
        b_q = 0
        t0 = time.perf_counter()
        for q in qs:
            t1 = time.perf_counter()
            idx.search_arrays(q, 10)
            lat.append(time.perf_counter() - t1)
        t_top = time.perf_counter() - t0
        idx.set_query_timing(True)
        dev_ms = 0.0
        for q in qs:
            idx.search_arrays(q, 10)
            dev_ms += idx.last_search_ms()[1]
        for q in qs:
            b_q += post_bytes(q) + 8 * 10
        # all hits (searcher.search(q, Integer.MAX_VALUE)): ordered on the device, copied to host arrays
        n_all = min(len(qs), 50)
        idx.search_all_arrays(qs[0])
        nh, all_dev, b_all = 0, 0.0, 0
        idx.set_query_timing(False)
        t0 = time.perf_counter()
        for q in qs[:n_all]:
            d, _ = idx.search_all_arrays(q)
            nh += len(d)
        t_all = time.perf_counter() - t0
        idx.set_query_timing(True)
        for q in qs[:n_all]:
            idx.search_all_arrays(q)
            all_dev += idx.last_search_ms()[1]
        for q in qs[:n_all]:
            b_all += post_bytes(q)
        b_all += 8 * nh
        # 16 request threads (Worker.processDocuments on Tomcat threads): each
        # search runs on the snapshot of the last commit with its own stream
        # and scratch, concurrently with the others (include/tfidf.h "Threading")
        import threading

        def threaded_qps(fn, per_thread, n_threads=16):
            bar = threading.Barrier(n_threads + 1)

            def body(t):
                bar.wait()
                for i in range(per_thread):
                    fn(qs[(t * per_thread + i) % len(qs)])
            th = [threading.Thread(target=body, args=(t,)) for t in range(n_threads)]
            for x in th:
                x.start()
            bar.wait()
            t0 = time.perf_counter()
            for x in th:
                x.join()
            return n_threads * per_thread / (time.perf_counter() - t0)

        idx.set_query_timing(False)
        threaded_qps(idx.search_all_arrays, 2)                      # contexts created
        mt_all = threaded_qps(idx.search_all_arrays, 25)
        mt_top = threaded_qps(lambda q: idx.search_arrays(q, 10), 100)
        idx.set_query_timing(True)
        bq = synth.queries(args.batch_queries)
        idx.search_batch(bq, 10)                                    # warm-up at full size (buffers sized)
        runs = []                                                   # median of 3 calls (device time)
        for _ in range(3):
            t0 = time.perf_counter()
            idx.search_batch(bq, 10)
            t_b = time.perf_counter() - t0
            runs.append((idx.last_search_ms()[1], idx.last_search_ms()[0], t_b))
        batch_runs_ms = [r[0] for r in runs]
        tot_ms, sc_ms, t_b = sorted(runs)[1]
        b_batch = min(sum(post_bytes(q) for q in bq), 8 * nnz + 9 * N) + 8 * 10 * len(bq)

        def roof(alg_bytes, ms):
            gbs = alg_bytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": gbs / HBM_PEAK_GBS, "alg_bytes": alg_bytes, "device_ms": ms}

        result["queries"] = {
            "single_top10_qps": len(qs) / t_top,
            "single_top10_p50_ms": float(np.percentile(lat, 50)) * 1e3,
            "single_top10_p99_ms": float(np.percentile(lat, 99)) * 1e3,
            "single_top10_device_ms_avg": dev_ms / len(qs),
            "single_all_hits_qps": n_all / t_all, "avg_hits": nh / n_all,
            "single_all_hits_device_ms_avg": all_dev / n_all,
            "threads16_all_hits_qps": mt_all, "threads16_top10_qps": mt_top,
            "batch10k_top10_qps": len(bq) / t_b,
            "batch10k_device_ms": tot_ms, "batch10k_scoring_ms": sc_ms, "batch10k_device_ms_runs": batch_runs_ms,
            "roofline": {
                "single_top10": roof(b_q / len(qs), dev_ms / len(qs)),
                "all_hits": roof(b_all / n_all, all_dev / n_all),
                "batch10k_top10": roof(b_batch, tot_ms),
                "note": "B_q = sum 9 df(t) + 8 k per query; all hits: sum 9 df(t) + 8 hits; "
                        "B_batch = min(sum_q sum_t 9 df(t), 8 nnz + 9 N) + 8 k Q (SURVEY §8(d)); "
                        "device time = HIP events on the index stream (scoring + ordering)"},
        }
    elif not args.no_queries:
        # node-level queries over the sharded corpus with GLOBAL statistics:
        # each rank scores every query on its shard, per-rank top-k keys are
        # all-gathered over RCCL and merged on device (tfidf_dist_search_batch)
        bq = synth.queries(args.batch_queries)
        adapter.search_batch(bq[:100], 10)
        out = {}
        for k in (10, 100):
            barrier()
            t0 = time.perf_counter()
            adapter.search_batch(bq, k)
            barrier()
            out["batch%dk_top%d_qps" % (len(bq) // 1000, k)] = len(bq) / (time.perf_counter() - t0)
        qs = synth.queries(max(args.queries, 1) // 4 or 1)
        lat = []
        for q in qs:
            barrier()
            t1 = time.perf_counter()
            adapter.search_arrays(q, 100)
            lat.append(time.perf_counter() - t1)
        out["single_top100_p50_ms"] = float(np.percentile(lat, 50)) * 1e3
        out["single_top100_qps"] = 1.0 / float(np.mean(lat))
        out["note"] = "node-level: %d ranks, GLOBAL stats, per-rank top-k all-gather + device merge" % world
        result["queries"] = out

    # ---- corpus loader: PCIe-inclusive end-to-end build (not `value`) ----
    if args.e2e and not dist_on:
        text, offs = corpus.to_host()
        best_add, best_tot = None, None
        for _ in range(2):
            idx.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            idx.add_documents_buffer(text, offs)
            t1 = time.perf_counter()
            idx.commit()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if best_tot is None or t2 - t0 < best_tot:
                best_add, best_tot = t1 - t0, t2 - t0
        result["end_to_end"] = {
            "docs_per_s": N / best_tot, "ms": best_tot * 1e3, "h2d_ms": best_add * 1e3,
            "h2d_GBs": len(text) / best_add / 1e9,
            "note": "host corpus (pageable numpy) -> pinned double-buffered staging -> HBM, then tfidf_commit; "
                    "best of 2"}
        del text, offs

    if rank == 0 and not dist_on and args.cpu_sample > 0:
        result["cpu_baseline"] = cpu_baseline(corpus, args, args.cpu_sample)
    corpus.free()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
    idx.close()


if __name__ == "__main__":
    main()
