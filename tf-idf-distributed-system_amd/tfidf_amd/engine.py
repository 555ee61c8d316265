"""ShardIndex: one GPU shard of the engine — the per-worker Lucene index of the
reference (Worker.java:54-55 ``luceneDir`` + ``indexWriter``) behind the C ABI.
"""
import ctypes as C
import os

import numpy as np

from . import _lib as L


def analyze(text: bytes):
    """StandardAnalyzer (Worker.java:71,225) as the engine runs it: lower-cased
    UTF-8 tokens of ``text`` (host side of the device scanner, unicode_scan.h)."""
    cap = 2 * len(text) + 64
    buf = C.create_string_buffer(cap)
    nt, nb = C.c_uint64(), C.c_uint64()
    L.check(L.load().tfidf_analyze(text, len(text), buf, cap, C.byref(nt), C.byref(nb)))
    return buf.raw[:nb.value].split(b"\0")[:nt.value]


def term_key(term: bytes):
    """128-bit device key (lo, hi) of an analysed (lower-cased) token."""
    lo, hi = C.c_uint64(), C.c_uint64()
    L.check(L.load().tfidf_term_key(term, len(term), C.byref(lo), C.byref(hi)))
    return lo.value, hi.value


class ShardIndex:
    def __init__(self, device=0, k1=1.2, b=0.75, vocab_capacity_log2=18, stats_mode=L.STATS_SHARD,
                 inversion=L.INVERSION_AUTO):
        lib = L.load()
        cfg = L.Config()
        L.check(lib.tfidf_config_init(C.byref(cfg)))
        cfg.k1, cfg.b, cfg.device = k1, b, device
        cfg.vocab_capacity_log2 = vocab_capacity_log2
        cfg.stats_mode = stats_mode
        cfg.inversion = inversion
        h = C.c_void_p()
        L.check(lib.tfidf_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self.device = device

    # -- lifetime -----------------------------------------------------------
    def close(self):
        if self._h:
            L.load().tfidf_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- indexing (Worker.addDocToIndex / IndexWriter.commit) ----------------
    def add_documents(self, texts, keys=None):
        """texts: list of bytes; keys: list of bytes (relative paths) or None."""
        n = len(texts)
        offs = np.zeros(n + 1, np.uint64)
        if n:
            offs[1:] = np.cumsum([len(t) for t in texts], dtype=np.uint64)
        blob = b"".join(texts)
        kb, koffs = None, None
        if keys is not None:
            assert len(keys) == n
            koffs = np.zeros(n + 1, np.uint64)
            if n:
                koffs[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64)
            kb = b"".join(keys)
        L.check(L.load().tfidf_add_docs(self._h, blob, L.ptr(offs, C.c_uint64), n, kb,
                                        None if koffs is None else L.ptr(koffs, C.c_uint64)))

    def add_documents_buffer(self, text, offsets):
        """Host corpus as one uint8 buffer + uint64 offsets[n + 1] (no per-doc
        Python objects): the loader path the reference's Worker.init feeds."""
        text = np.ascontiguousarray(text, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        L.check(L.load().tfidf_add_docs(self._h, C.c_void_p(text.ctypes.data), L.ptr(offsets, C.c_uint64),
                                        len(offsets) - 1, None, None))

    def save(self, path):
        """Persist the staged corpus + keys (tfidf_save); the index is rebuilt by commit() after load()."""
        L.check(L.load().tfidf_save(self._h, os.fsencode(path)))

    def load(self, path):
        """Stage a saved index file into this (empty) index; call commit() next."""
        L.check(L.load().tfidf_load(self._h, os.fsencode(path)))

    def clear(self):
        """Drop all staged/committed documents; device buffers are kept for reuse."""
        L.check(L.load().tfidf_clear(self._h))

    def add_documents_device(self, d_text, d_offsets, n_docs, total_bytes):
        L.check(L.load().tfidf_add_docs_device(self._h, C.c_void_p(d_text), C.c_void_p(d_offsets), n_docs,
                                               total_bytes))

    def commit(self):
        L.check(L.load().tfidf_commit(self._h))

    def set_hash_attempt(self, attempt):
        """Seed attempt (0..3) the following commits start from (tfidf_set_hash_attempt)."""
        L.check(L.load().tfidf_set_hash_attempt(self._h, attempt))

    def commit_timing(self):
        t = L.CommitTiming()
        L.check(L.load().tfidf_get_commit_timing(self._h, C.byref(t)))
        return {f: getattr(t, f) for f, _ in L.CommitTiming._fields_}

    def stats(self):
        s = L.IndexStats()
        L.check(L.load().tfidf_stats(self._h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in L.IndexStats._fields_}

    # -- search (Worker.searchIndex) ------------------------------------------
    def search(self, query: bytes, k=0):
        """[(doc, float score)] in (score desc, doc asc); k == 0 -> all hits."""
        if k == 0:                              # sized by the snapshot the search runs on
            with self.reader() as rd:
                return rd.search(query, 0)
        lib = L.load()
        docs = np.zeros(k, np.uint32)
        scores = np.zeros(k, np.float32)
        n = C.c_uint64()
        rc = lib.tfidf_search(self._h, query, len(query), k, L.ptr(docs, C.c_uint32), L.ptr(scores, C.c_float),
                              k, C.byref(n))
        L.check(rc)
        m = n.value
        return list(zip(docs[:m].tolist(), scores[:m].tolist()))

    def reader(self):
        """A Reader on the snapshot published now (tfidf_reader_open)."""
        return Reader(self)

    def search_coalesced(self, query: bytes, k, wait_us=50):
        """Thread-safe top-k search that shares one batched scoring launch with
        the searches other threads issue at the same time (tfidf_search_coalesced)."""
        docs = np.zeros(k, np.uint32)
        scores = np.zeros(k, np.float32)
        n = C.c_uint64()
        L.check(L.load().tfidf_search_coalesced(self._h, query, len(query), k, L.ptr(docs, C.c_uint32),
                                                L.ptr(scores, C.c_float), k, C.byref(n), wait_us))
        m = n.value
        return list(zip(docs[:m].tolist(), scores[:m].tolist()))

    def search_all_arrays(self, query: bytes):
        """All hits as (doc uint32[], score float32[]) in (score desc, doc asc)
        — searcher.search(q, Integer.MAX_VALUE) without per-hit Python objects."""
        with self.reader() as rd:
            return rd.search_arrays(query, 0)

    def search_arrays(self, query: bytes, k):
        lib = L.load()
        docs = np.zeros(max(k, 1), np.uint32)
        scores = np.zeros(max(k, 1), np.float32)
        n = C.c_uint64()
        L.check(lib.tfidf_search(self._h, query, len(query), k, L.ptr(docs, C.c_uint32), L.ptr(scores, C.c_float),
                                 max(k, 1), C.byref(n)))
        return docs[:n.value], scores[:n.value]

    def search_batch(self, queries, k):
        """queries: list of bytes.  Returns (docs[n_q, k], scores[n_q, k], counts[n_q])."""
        nq = len(queries)
        offs = np.zeros(nq + 1, np.uint64)
        offs[1:] = np.cumsum([len(q) for q in queries], dtype=np.uint64)
        docs = np.zeros((nq, k), np.uint32)
        scores = np.zeros((nq, k), np.float32)
        counts = np.zeros(nq, np.uint32)
        L.check(L.load().tfidf_search_batch(self._h, b"".join(queries), L.ptr(offs, C.c_uint64), nq, k,
                                            L.ptr(docs, C.c_uint32), L.ptr(scores, C.c_float),
                                            L.ptr(counts, C.c_uint32)))
        return docs, scores, counts

    def search_batch_keys_device(self, queries, k, doc_base, d_keys):
        """n_q x k merge keys (score bits << 32 | ~(doc_base + doc)) into device memory d_keys."""
        nq = len(queries)
        offs = np.zeros(nq + 1, np.uint64)
        offs[1:] = np.cumsum([len(q) for q in queries], dtype=np.uint64)
        L.check(L.load().tfidf_search_batch_keys_device(self._h, b"".join(queries), L.ptr(offs, C.c_uint64), nq, k,
                                                        doc_base, C.c_void_p(d_keys)))

    def search_all_keys_device(self, query: bytes, doc_base, d_keys, cap):
        """Every hit's merge key, ordered, into device memory (cap >= num_docs); -> #hits."""
        n = C.c_uint64()
        L.check(L.load().tfidf_search_all_keys_device(self._h, query, len(query), doc_base, C.c_void_p(d_keys), cap,
                                                      C.byref(n)))
        return n.value

    def set_stream(self, stream):
        """Issue device work on the caller's HIP stream (int handle); None = the index's own stream."""
        L.check(L.load().tfidf_set_stream(self._h, L.OWN_STREAM if stream is None else C.c_void_p(stream)))

    def set_query_timing(self, on: bool):
        """HIP-event device timing of searches (on by default; off for serving)."""
        L.check(L.load().tfidf_set_query_timing(self._h, 1 if on else 0))

    def last_search_ms(self):
        a, b = C.c_float(), C.c_float()
        L.check(L.load().tfidf_last_search_ms(self._h, C.byref(a), C.byref(b)))
        return a.value, b.value

    # -- inspection -----------------------------------------------------------
    def doc_key(self, doc):
        buf = C.create_string_buffer(4096)
        n = C.c_uint64()
        L.check(L.load().tfidf_doc_key(self._h, doc, buf, 4096, C.byref(n)))
        return buf.raw[:n.value]

    def doc_keys(self):
        """Every committed document's key: (uint8 blob, uint64 offsets[num_docs + 1])."""
        with self.reader() as rd:
            return rd.doc_keys()

    def malformed_docs(self):
        """Committed doc ids whose bytes are not valid UTF-8 (indexed empty)."""
        n = self.stats()["malformed_docs"]
        out = np.zeros(max(n, 1), np.uint64)
        m = C.c_uint64()
        L.check(L.load().tfidf_malformed_docs(self._h, L.ptr(out, C.c_uint64), len(out), C.byref(m)))
        return out[:m.value].tolist()

    def doc_len(self, doc):
        ln, nm = C.c_uint32(), C.c_uint8()
        L.check(L.load().tfidf_doc_len(self._h, doc, C.byref(ln), C.byref(nm)))
        return ln.value, nm.value

    def doc_terms(self, doc):
        ln, _ = self.doc_len(doc)
        cap = ln + 1
        tfs = np.zeros(cap, np.uint32)
        n = C.c_uint64()
        for per in (48, 1024):                   # term strings: up to 255 UTF-16 units (<= 1020 bytes)
            buf = C.create_string_buffer(cap * per + 64)
            rc = L.load().tfidf_doc_terms(self._h, doc, buf, len(buf), L.ptr(tfs, C.c_uint32), cap, C.byref(n))
            if rc != L.E_BUFFER:
                break
        L.check(rc)
        terms = buf.raw.split(b"\0")[:n.value]
        return dict(zip(terms, tfs[:n.value].tolist()))

    def df(self, term: bytes):
        a, b = C.c_uint64(), C.c_uint64()
        L.check(L.load().tfidf_term_df(self._h, term, len(term), C.byref(a), C.byref(b)))
        return a.value, b.value

    # -- GLOBAL statistics ------------------------------------------------------
    def vocab_size(self):
        n = C.c_uint64()
        L.check(L.load().tfidf_vocab_size(self._h, C.byref(n)))
        return n.value

    def vocab_export(self):
        """(keys uint64 [n, 2] (lo, hi) sorted by (hi, lo), df_local uint32 [n],
        df_effective uint32 [n]): the vocabulary with the statistics in force."""
        n = self.vocab_size()
        keys = np.zeros((max(n, 1), 2), np.uint64)
        dl = np.zeros(max(n, 1), np.uint32)
        de = np.zeros(max(n, 1), np.uint32)
        m = C.c_uint64()
        L.check(L.load().tfidf_vocab_export(self._h, L.ptr(keys, C.c_uint64), L.ptr(dl, C.c_uint32),
                                            L.ptr(de, C.c_uint32), len(dl), C.byref(m)))
        return keys[:m.value], dl[:m.value], de[:m.value]

    def vocab_export_device(self, d_keys, d_df, cap):
        n = C.c_uint64()
        L.check(L.load().tfidf_vocab_export_device(self._h, C.c_void_p(d_keys), C.c_void_p(d_df), cap, C.byref(n)))
        return n.value

    def vocab_canonicalize_device(self, d_all_keys, n_all, d_df_canon, cap):
        n = C.c_uint64()
        L.check(L.load().tfidf_vocab_canonicalize_device(self._h, C.c_void_p(d_all_keys), n_all,
                                                         C.c_void_p(d_df_canon), cap, C.byref(n)))
        return n.value

    def set_global_stats_device(self, d_df_canon, n_canon, doc_count, sum_ttf):
        L.check(L.load().tfidf_set_global_stats_device(self._h, C.c_void_p(d_df_canon), n_canon, doc_count,
                                                       sum_ttf))

    def vocab_partition_device(self, n_ranks, d_records, cap, d_counts):
        """Records (lo, hi, df) grouped by owner rank into d_records, per-owner
        counts (u64) into d_counts -> n records.  Asynchronous on a stream set
        by set_stream (the buffers must then stay live until that stream
        reaches the work: torch tensors of that stream do); on the index's own
        stream it returns with the work done."""
        n = C.c_uint64()
        L.check(L.load().tfidf_vocab_partition_device(self._h, n_ranks, C.c_void_p(d_records), cap,
                                                      C.c_void_p(d_counts), C.byref(n)))
        return n.value

    def vocab_reduce_device(self, d_records, n, d_df_out, d_n_unique=None):
        """Owner side: summed df per received record (asynchronous on a
        set_stream stream, like vocab_partition_device)."""
        L.check(L.load().tfidf_vocab_reduce_device(self._h, C.c_void_p(d_records), n, C.c_void_p(d_df_out),
                                                   C.c_void_p(d_n_unique) if d_n_unique else None))

    def set_global_df_device(self, d_df, n, doc_count, sum_ttf):
        L.check(L.load().tfidf_set_global_df_device(self._h, C.c_void_p(d_df), n, doc_count, sum_ttf))

    def set_global_stats(self, keys_lohi, df, doc_count, sum_ttf):
        keys_lohi = np.ascontiguousarray(keys_lohi, np.uint64).reshape(-1)
        df = np.ascontiguousarray(df, np.uint64)
        L.check(L.load().tfidf_set_global_stats(self._h, L.ptr(keys_lohi, C.c_uint64), L.ptr(df, C.c_uint64),
                                                len(df), doc_count, sum_ttf))

    def clear_global_stats(self):
        L.check(L.load().tfidf_clear_global_stats(self._h))


def sort_names(blob, offsets):
    """Permutation of the names blob[offsets[i]:offsets[i+1]] in String.compareTo order."""
    n = len(offsets) - 1
    blob = np.ascontiguousarray(blob, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    perm = np.zeros(max(n, 1), np.uint64)
    L.check(L.load().tfidf_sort_names(blob.tobytes(), L.ptr(offsets, C.c_uint64), n, L.ptr(perm, C.c_uint64)))
    return perm[:n]


def leader_merge(responses):
    """Leader.start merge via the C ABI: list (worker order) of lists of
    (name bytes, double) -> [(name, sum)] ordered by name."""
    flat = [x for r in responses for x in r]
    n = len(flat)
    if n == 0:
        return []
    names = b"".join(nm for nm, _ in flat)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(nm) for nm, _ in flat], dtype=np.uint64)
    sc = np.array([s for _, s in flat], np.float64)
    first = np.zeros(n, np.uint64)
    sums = np.zeros(n, np.float64)
    m = C.c_uint64()
    L.check(L.load().tfidf_leader_merge(names, L.ptr(offs, C.c_uint64), n, L.ptr(sc, C.c_double),
                                        L.ptr(first, C.c_uint64), L.ptr(sums, C.c_double), C.byref(m)))
    return [(flat[int(first[i])][0], float(sums[i])) for i in range(m.value)]


class Reader:
    """A pinned snapshot (tfidf_reader_*): Worker.java:223 opens a
    DirectoryReader on the last commit per request and reads the hits' stored
    "path" from it (:234-238); searches and doc keys here all see the commit
    published when the reader was opened, whatever commits follow."""

    def __init__(self, index):
        self._h = C.c_void_p()
        L.check(L.load().tfidf_reader_open(index._h, C.byref(self._h)))
        g, n = C.c_uint64(), C.c_uint64()
        L.check(L.load().tfidf_reader_info(self._h, C.byref(g), C.byref(n)))
        self.generation, self.num_docs = g.value, n.value

    def close(self):
        if self._h:
            L.load().tfidf_reader_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def search_arrays(self, query: bytes, k=0):
        cap = max(k if k else self.num_docs, 1)
        docs = np.empty(cap, np.uint32)
        scores = np.empty(cap, np.float32)
        n = C.c_uint64()
        L.check(L.load().tfidf_reader_search(self._h, query, len(query), k, L.ptr(docs, C.c_uint32),
                                             L.ptr(scores, C.c_float), cap, C.byref(n)))
        return docs[:n.value], scores[:n.value]

    def search(self, query: bytes, k=0):
        d, s = self.search_arrays(query, k)
        return list(zip(d.tolist(), s.tolist()))

    def doc_key(self, doc):
        buf = C.create_string_buffer(4096)
        n = C.c_uint64()
        L.check(L.load().tfidf_reader_doc_key(self._h, doc, buf, 4096, C.byref(n)))
        return buf.raw[:n.value]

    def doc_keys(self):
        lib = L.load()
        offs = np.zeros(self.num_docs + 1, np.uint64)
        need = C.c_uint64()
        rc = lib.tfidf_reader_doc_keys(self._h, None, 0, L.ptr(offs, C.c_uint64), C.byref(need))
        if rc not in (L.OK, L.E_BUFFER):
            L.check(rc)
        buf = C.create_string_buffer(max(need.value, 1))
        L.check(lib.tfidf_reader_doc_keys(self._h, buf, need.value, L.ptr(offs, C.c_uint64), C.byref(need)))
        return np.frombuffer(buf.raw[:need.value], np.uint8).copy(), offs
