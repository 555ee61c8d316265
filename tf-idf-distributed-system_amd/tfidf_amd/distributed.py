"""Node-level search over GPU shards: a thin ctypes layer over libtfidf's
node-level C ABI (include/tfidf.h, "Node level").  The orchestration itself —
GLOBAL statistics by term ownership, hash-seed agreement, top-k / all-hits /
batch merges of device merge keys, SHARD mode's name table and Leader-style
merge — is C++ in the library (csrc/tfidf_dist.hip), the same code a Java host
reaches over JNI.  It replaces the reference's
Leader.start fan-out + merge (Leader.java:39-92) over Worker.searchIndex
(Worker.java:222-241) with collectives between GPU shards.

Transports of a Comm (one per rank, one process per GPU):
  * "rccl": the library's built-in RCCL communicator (over xGMI on MI355X);
    the 128-byte unique id travels over the torch.distributed group.
  * "callback": the group's own collectives (gloo, host memory) passed to the
    library as C callbacks (tfidf_collectives) — the CPU tests and several
    ranks sharing one GPU.
Node: one process owning a device list (tfidf_node_*).

Two modes:
  * GLOBAL (the reference's 1-worker results on a sharded corpus): exchanged
    docFreq / docCount / sumTotalTermFreq, global doc ids = shard base + local.
  * SHARD (the reference's N workers, Leader.java:39-92): each rank scores with
    its own statistics; every hit summed per document name in rank order
    (Double::sum), ordered by name (TreeMap, String.compareTo).
"""
import ctypes as C

import numpy as np

from . import _lib as L

# A query that does not parse (QueryParser ParseException / TooManyClauses) or
# is not valid UTF-8: the reference's Worker answers [] (Worker.java:182-185),
# so its Leader merges nothing.  Every rank fails alike, before any collective.
QUERY_ERRORS = (L.QuerySyntaxError, L.UnsupportedQuery)

AG_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)
A2A_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p,
                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p)


class Collectives(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("memory", C.c_int32), ("all_gather", AG_FN), ("all_to_all_v", A2A_FN)]


def _host_view(addr, n):
    return np.ctypeslib.as_array((C.c_uint8 * n).from_address(addr)) if n else np.zeros(0, np.uint8)


def torch_host_collectives(group=None):
    """tfidf_collectives over a torch.distributed group on host tensors (gloo):
    the library stages device data through host memory around each call."""
    import torch
    import torch.distributed as dist

    ws = dist.get_world_size(group)

    def all_gather(ctx, send, recv, nbytes, stream):
        try:
            src = torch.from_numpy(_host_view(send, nbytes).copy())
            parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(ws)]
            dist.all_gather(parts, src, group=group)
            _host_view(recv, nbytes * ws)[:] = torch.cat(parts).numpy()
            return 0
        except Exception:                               # an exception must not cross the C frames
            return 1

    def all_to_all_v(ctx, send, sb, so, recv, rb, ro, stream):
        try:
            sbl = [int(sb[r]) for r in range(ws)]
            rbl = [int(rb[r]) for r in range(ws)]
            inp = np.concatenate([_host_view(send + int(so[r]), sbl[r]) if sbl[r] else np.zeros(0, np.uint8)
                                  for r in range(ws)]) if send else np.zeros(sum(sbl), np.uint8)
            out = torch.empty(sum(rbl), dtype=torch.uint8)
            dist.all_to_all_single(out, torch.from_numpy(np.ascontiguousarray(inp)), output_split_sizes=rbl,
                                   input_split_sizes=sbl, group=group)
            o = out.numpy()
            at = 0
            for r in range(ws):
                if rbl[r]:
                    _host_view(recv + int(ro[r]), rbl[r])[:] = o[at:at + rbl[r]]
                at += rbl[r]
            return 0
        except Exception:
            return 1

    return all_gather, all_to_all_v


class Comm:
    """A tfidf_comm (one rank of a communicator)."""

    def __init__(self, handle, keep=()):
        self._h = handle
        self._keep = keep                                # ctypes callbacks must outlive the communicator

    @classmethod
    def from_group(cls, group=None, device=0, transport="auto"):
        """Communicator over a torch.distributed group: the built-in RCCL one
        ("rccl"; default when the group's backend is nccl) or the group's
        collectives as host callbacks ("callback"; default for gloo)."""
        import torch.distributed as dist
        lib = L.load()
        rank, ws = dist.get_rank(group), dist.get_world_size(group)
        if transport == "auto":
            transport = "rccl" if dist.get_backend(group) == "nccl" else "callback"
        h = C.c_void_p()
        if transport == "rccl":
            uid = (C.c_uint8 * 128)()
            if rank == 0:
                L.check(lib.tfidf_rccl_unique_id(uid))
            box = [bytes(uid)]
            dist.broadcast_object_list(box, src=0, group=group)
            uid = (C.c_uint8 * 128).from_buffer_copy(box[0])
            L.check(lib.tfidf_comm_init_rccl(uid, rank, ws, device, C.byref(h)))
            return cls(h)
        ag, a2a = torch_host_collectives(group)
        cag, ca2a = AG_FN(ag), A2A_FN(a2a)
        coll = Collectives(None, 0, cag, ca2a)
        L.check(lib.tfidf_comm_create(rank, ws, C.byref(coll), C.byref(h)))
        return cls(h, keep=(cag, ca2a))

    @classmethod
    def inproc(cls, world):
        """`world` communicators of this process (one thread per rank)."""
        arr = (C.c_void_p * world)()
        L.check(L.load().tfidf_comm_create_inproc(world, arr))
        return [cls(C.c_void_p(arr[i])) for i in range(world)]

    def info(self):
        r, w, t = C.c_int32(), C.c_int32(), C.c_int32()
        L.check(L.load().tfidf_comm_info(self._h, C.byref(r), C.byref(w), C.byref(t)))
        return r.value, w.value, {0: "callback", 1: "rccl", 2: "inproc"}[t.value]

    def selftest(self):
        L.check(L.load().tfidf_comm_selftest(self._h))

    def close(self):
        if self._h:
            L.load().tfidf_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _offsets(items):
    offs = np.zeros(len(items) + 1, np.uint64)
    if items:
        offs[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    return offs


class DistShard:
    """One rank's shard in process model (2): every method is collective
    (every rank calls it, in the same order)."""

    def __init__(self, shard, comm, doc_base=0):
        self.shard = shard
        self.comm = comm
        self.doc_base = doc_base

    # -- statistics -----------------------------------------------------------
    def global_commit(self, vocab_size=False):
        """GLOBAL statistics (after this rank's own commit) -> (global
        vocabulary size or None, docCount, sumTTF)."""
        nv, dc, ttf = C.c_uint64(), C.c_uint64(), C.c_uint64()
        L.check(L.load().tfidf_dist_global_commit(self.shard._h, self.comm._h, C.byref(nv) if vocab_size else None,
                                                  C.byref(dc), C.byref(ttf)))
        return (nv.value if vocab_size else None), dc.value, ttf.value

    def shard_commit(self):
        """SHARD mode name table (once per commit) -> distinct names over all ranks."""
        n = C.c_uint64()
        L.check(L.load().tfidf_dist_shard_commit(self.shard._h, self.comm._h, C.byref(n)))
        return n.value

    # -- GLOBAL search ------------------------------------------------------------
    def search_arrays(self, query: bytes, k):
        """(global doc int64[], score float32[]) in (score desc, doc asc);
        k == 0: every hit; [] for a query that does not parse."""
        lib = L.load()
        cap = max(k, 1) if k else 1 << 16
        docs = np.zeros(cap, np.uint64)
        scores = np.zeros(cap, np.float32)
        n = C.c_uint64()
        try:
            rc = lib.tfidf_dist_search(self.shard._h, self.comm._h, self.doc_base, query, len(query), k,
                                       L.ptr(docs, C.c_uint64), L.ptr(scores, C.c_float), cap, C.byref(n))
            if rc == L.E_BUFFER:
                docs = np.zeros(n.value, np.uint64)
                scores = np.zeros(n.value, np.float32)
                rc = lib.tfidf_dist_last_hits(self.comm._h, L.ptr(docs, C.c_uint64), L.ptr(scores, C.c_float),
                                              n.value, C.byref(n))
            L.check(rc)
        except QUERY_ERRORS:
            return np.zeros(0, np.int64), np.zeros(0, np.float32)
        return docs[:n.value].astype(np.int64), scores[:n.value]

    def search(self, query: bytes, k):
        d, s = self.search_arrays(query, k)
        return list(zip(d.tolist(), s.tolist()))

    def search_batch(self, queries, k):
        """(docs int64[n_q, k], scores float32[n_q, k], counts int64[n_q]), global doc ids."""
        nq = len(queries)
        offs = _offsets(queries)
        docs = np.zeros((nq, k), np.uint64)
        scores = np.zeros((nq, k), np.float32)
        counts = np.zeros(nq, np.uint32)
        L.check(L.load().tfidf_dist_search_batch(self.shard._h, self.comm._h, self.doc_base, b"".join(queries),
                                                 L.ptr(offs, C.c_uint64), nq, k, L.ptr(docs, C.c_uint64),
                                                 L.ptr(scores, C.c_float), L.ptr(counts, C.c_uint32)))
        return docs.astype(np.int64), scores, counts.astype(np.int64)

    # -- SHARD search (Leader.start) ------------------------------------------------
    def shard_search(self, query: bytes):
        """[(name bytes, double)] in String.compareTo order."""
        n, nb = C.c_uint64(), C.c_uint64()
        try:
            L.check(L.load().tfidf_dist_shard_search(self.shard._h, self.comm._h, query, len(query), C.byref(n),
                                                     C.byref(nb)))
        except QUERY_ERRORS:
            return []
        return _last_names(self.comm._h, n.value, nb.value)


    def last_failed(self):
        """Ranks skipped by the last shard_search (bit r = rank r)."""
        m = C.c_uint64()
        L.check(L.load().tfidf_dist_last_failed(self.comm._h, C.byref(m)))
        return m.value


def _last_names(h, n, nb):
    buf = C.create_string_buffer(max(nb, 1))
    offs = np.zeros(n + 1, np.uint64)
    sc = np.zeros(max(n, 1), np.float64)
    m, b = C.c_uint64(), C.c_uint64()
    L.check(L.load().tfidf_dist_last_names(h, buf, max(nb, 1), L.ptr(offs, C.c_uint64), L.ptr(sc, C.c_double),
                                           n, C.byref(m), C.byref(b)))
    raw = buf.raw
    return [(raw[int(offs[i]):int(offs[i + 1])], float(sc[i])) for i in range(m.value)]


class Node:
    """Process model (1): one process, one shard per device (tfidf_node_*)."""

    def __init__(self, devices=(0,), stats_mode=L.STATS_GLOBAL, inproc=False, vocab_capacity_log2=18,
                 inversion=L.INVERSION_AUTO):
        lib = L.load()
        cfg = L.Config()
        L.check(lib.tfidf_config_init(C.byref(cfg)))
        cfg.stats_mode = stats_mode
        cfg.vocab_capacity_log2 = vocab_capacity_log2
        cfg.inversion = inversion
        dev = (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        L.check(lib.tfidf_node_create_devices(C.byref(cfg), dev, len(devices), 1 if inproc else 0, C.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            L.load().tfidf_node_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_documents(self, texts, keys=None, shard=-1):
        offs = _offsets(texts)
        koffs = _offsets(keys) if keys is not None else None
        L.check(L.load().tfidf_node_add_docs(self._h, shard, b"".join(texts), L.ptr(offs, C.c_uint64), len(texts),
                                             b"".join(keys) if keys is not None else None,
                                             L.ptr(koffs, C.c_uint64) if keys is not None else None))

    def commit(self):
        L.check(L.load().tfidf_node_commit(self._h))

    def stats(self):
        s = NodeStats()
        L.check(L.load().tfidf_node_stats_get(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in NodeStats._fields_}

    def search(self, query: bytes, k):
        lib = L.load()
        cap = max(k, 1) if k else max(self.stats()["num_docs"], 1)
        docs = np.zeros(cap, np.uint64)
        scores = np.zeros(cap, np.float32)
        n = C.c_uint64()
        try:
            L.check(lib.tfidf_node_search(self._h, query, len(query), k, L.ptr(docs, C.c_uint64),
                                          L.ptr(scores, C.c_float), cap, C.byref(n)))
        except QUERY_ERRORS:
            return []
        return list(zip(docs[:n.value].astype(np.int64).tolist(), scores[:n.value].tolist()))

    def search_batch(self, queries, k):
        nq = len(queries)
        offs = _offsets(queries)
        docs = np.zeros((nq, k), np.uint64)
        scores = np.zeros((nq, k), np.float32)
        counts = np.zeros(nq, np.uint32)
        L.check(L.load().tfidf_node_search_batch(self._h, b"".join(queries), L.ptr(offs, C.c_uint64), nq, k,
                                                 L.ptr(docs, C.c_uint64), L.ptr(scores, C.c_float),
                                                 L.ptr(counts, C.c_uint32)))
        return docs.astype(np.int64), scores, counts.astype(np.int64)

    def search_names(self, query: bytes):
        lib = L.load()
        n, nb = C.c_uint64(), C.c_uint64()
        try:
            rc = lib.tfidf_node_search_names(self._h, query, len(query), None, 0, None, None, 0, C.byref(n), C.byref(nb))
            if rc != L.E_BUFFER:
                L.check(rc)
            if n.value == 0:
                return []
        except QUERY_ERRORS:
            return []
        buf = C.create_string_buffer(max(nb.value, 1))
        offs = np.zeros(n.value + 1, np.uint64)
        sc = np.zeros(n.value, np.float64)
        L.check(lib.tfidf_node_search_names(self._h, query, len(query), buf, nb.value, L.ptr(offs, C.c_uint64),
                                            L.ptr(sc, C.c_double), n.value, C.byref(n), C.byref(nb)))
        raw = buf.raw
        return [(raw[int(offs[i]):int(offs[i + 1])], float(sc[i])) for i in range(n.value)]

    def last_failed(self):
        """Shards skipped by the last search_names (bit g = shard g)."""
        m = C.c_uint64()
        L.check(L.load().tfidf_node_last_failed(self._h, C.byref(m)))
        return m.value

    def shard(self, i):
        """Shard i's tfidf_index handle (owned by the node)."""
        h = C.c_void_p()
        L.check(L.load().tfidf_node_shard(self._h, i, C.byref(h), None))
        return h

    def doc_key(self, doc):
        buf = C.create_string_buffer(4096)
        n = C.c_uint64()
        L.check(L.load().tfidf_node_doc_key(self._h, doc, buf, 4096, C.byref(n)))
        return buf.raw[:n.value]


class NodeStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("n_shards", "num_docs", "doc_count", "sum_ttf", "num_terms", "transport")]


def shard_range(n_docs, rank, world):
    """Contiguous document range of a rank: [rank*N/G, (rank+1)*N/G)."""
    return rank * n_docs // world, (rank + 1) * n_docs // world
