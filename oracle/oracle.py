"""ctypes wrapper of the CPU ORACLE (oracle/liboracle.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It restates Lucene 9.8.0's StandardAnalyzer + BM25Similarity as
called from Worker.java:190-241 and the Leader.java:73-88 merge; see
tfidf_oracle.h for the full citation list and what pins it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

OK, E_ARG, E_UNSUPPORTED, E_NOMEM, E_CAP, E_SYNTAX = 0, -1, -2, -3, -4, -5


class QuerySyntaxError(ValueError):
    """QueryParser ParseException / TooManyClauses (the reference answers [])."""


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    u8p, u32p, u64p, f32p, f64p = (C.POINTER(C.c_uint8), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_float),
                                   C.POINTER(C.c_double))
    sig = {
        "orc_tokenize": (C.c_int64, [C.c_char_p, C.c_uint64, C.c_uint32, u32p, u32p, C.c_uint64]),
        "orc_tokenize_unicode": (C.c_int64, [C.c_char_p, C.c_uint64, C.c_uint32, u32p, u32p, C.c_uint64]),
        "orc_lower_utf8": (C.c_uint64, [C.c_char_p, C.c_uint64, C.c_char_p]),
        "orc_int_to_byte4": (C.c_uint8, [C.c_int32]),
        "orc_byte4_to_int": (C.c_int32, [C.c_uint8]),
        "orc_create": (C.c_void_p, [C.c_float, C.c_float]),
        "orc_destroy": (None, [C.c_void_p]),
        "orc_add_doc": (C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64]),
        "orc_commit": (C.c_int, [C.c_void_p]),
        "orc_num_docs": (C.c_uint64, [C.c_void_p]),
        "orc_doc_count": (C.c_uint64, [C.c_void_p]),
        "orc_sum_ttf": (C.c_uint64, [C.c_void_p]),
        "orc_num_terms": (C.c_uint64, [C.c_void_p]),
        "orc_doc_len": (C.c_uint32, [C.c_void_p, C.c_uint64]),
        "orc_malformed_docs": (C.c_uint64, [C.c_void_p, u64p, C.c_uint64]),
        "orc_doc_norm": (C.c_uint8, [C.c_void_p, C.c_uint64]),
        "orc_doc_key": (C.c_uint64, [C.c_void_p, C.c_uint64, C.c_char_p, C.c_uint64]),
        "orc_doc_terms": (C.c_int64, [C.c_void_p, C.c_uint64, C.c_char_p, C.c_uint64, u32p, C.c_uint64]),
        "orc_df": (C.c_int64, [C.c_void_p, C.c_char_p, C.c_uint64]),
        "orc_vocab": (C.c_int64, [C.c_void_p, C.c_char_p, C.c_uint64, u32p, C.c_uint64]),
        "orc_set_global_stats": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64]),
        "orc_set_global_df": (C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint64]),
        "orc_search": (C.c_int, [C.c_void_p, C.c_char_p, C.c_uint64, C.c_uint32, u32p, f32p, C.c_uint64, u64p]),
        "orc_query_terms": (C.c_int64, [C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64, f32p, C.c_uint64]),
        "orc_idf": (C.c_float, [C.c_uint64, C.c_uint64]),
        "orc_avgdl": (C.c_float, [C.c_uint64, C.c_uint64]),
        "orc_norm_cache": (None, [C.c_float, C.c_float, C.c_float, f32p]),
        "orc_bm25": (C.c_float, [C.c_float, C.c_uint32, C.c_float]),
        "orc_leader_merge": (C.c_int64, [C.c_char_p, u64p, C.c_uint64, f64p, u64p, f64p]),
        "orc_bulk_build": (C.c_int, [C.c_void_p, u64p, C.c_uint64, C.c_uint32, f64p, u64p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def lower_utf8(tok: bytes) -> bytes:
    """LowerCaseFilter of one token (JDK 17 Character.toLowerCase per code point)."""
    out = C.create_string_buffer(2 * len(tok) + 8)
    n = lib().orc_lower_utf8(tok, len(tok), out)
    return out.raw[:n]


def tokenize(text: bytes, max_len=255, force_unicode=False):
    """Token byte strings (lower-cased) of ``text``; raises on malformed UTF-8.
    ASCII text takes the oracle's byte-rule path unless force_unicode."""
    cap = len(text) // 2 + 2
    st = np.zeros(cap, np.uint32)
    ln = np.zeros(cap, np.uint32)
    f = lib().orc_tokenize_unicode if force_unicode else lib().orc_tokenize
    n = f(text, len(text), max_len, _p(st, C.c_uint32), _p(ln, C.c_uint32), cap)
    if n < 0:
        raise ValueError("unsupported input (malformed UTF-8)")
    return [lower_utf8(text[s:s + l]) for s, l in zip(st[:n], ln[:n])]


def int_to_byte4(i):
    return lib().orc_int_to_byte4(i)


def byte4_to_int(b):
    return lib().orc_byte4_to_int(b)


def query_terms(q: bytes):
    cap = len(q) // 2 + 2
    buf = C.create_string_buffer(len(q) + cap + 16)
    boosts = np.zeros(cap, np.float32)
    n = lib().orc_query_terms(q, len(q), buf, len(buf), _p(boosts, C.c_float), cap)
    if n == E_SYNTAX:
        raise QuerySyntaxError("query does not parse")
    if n < 0:
        raise ValueError("query rejected: %d" % n)
    terms = buf.raw.split(b"\0")[:n]
    return list(zip(terms, boosts[:n].tolist()))


class OracleIndex:
    """One shard (one reference Worker) restated on the CPU."""

    def __init__(self, k1=1.2, b=0.75):
        self._ix = lib().orc_create(k1, b)
        self.k1, self.b = k1, b

    def close(self):
        if self._ix:
            lib().orc_destroy(self._ix)
            self._ix = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_doc(self, key: bytes, text: bytes):
        rc = lib().orc_add_doc(self._ix, key, len(key), text, len(text))
        if rc != OK:
            raise RuntimeError("orc_add_doc rc=%d" % rc)

    def commit(self):
        rc = lib().orc_commit(self._ix)
        if rc != OK:
            raise ValueError("orc_commit rc=%d" % rc)

    @property
    def num_docs(self):
        return lib().orc_num_docs(self._ix)

    @property
    def doc_count(self):
        return lib().orc_doc_count(self._ix)

    @property
    def sum_ttf(self):
        return lib().orc_sum_ttf(self._ix)

    @property
    def num_terms(self):
        return lib().orc_num_terms(self._ix)

    def doc_len(self, d):
        return lib().orc_doc_len(self._ix, d)

    def malformed_docs(self):
        n = lib().orc_malformed_docs(self._ix, None, 0)
        out = np.zeros(max(n, 1), np.uint64)
        lib().orc_malformed_docs(self._ix, _p(out, C.c_uint64), n)
        return out[:n].tolist()

    def doc_norm(self, d):
        return lib().orc_doc_norm(self._ix, d)

    def doc_key(self, d):
        buf = C.create_string_buffer(4096)
        n = lib().orc_doc_key(self._ix, d, buf, 4096)
        return buf.raw[:n]

    def doc_terms(self, d):
        """{term bytes: tf} for doc d."""
        cap = self.doc_len(d) + 1
        buf = C.create_string_buffer(cap * 260 + 16)
        tfs = np.zeros(cap, np.uint32)
        n = lib().orc_doc_terms(self._ix, d, buf, len(buf), _p(tfs, C.c_uint32), cap)
        if n < 0:
            raise RuntimeError("orc_doc_terms rc=%d" % n)
        terms = buf.raw.split(b"\0")[:n]
        return dict(zip(terms, tfs[:n].tolist()))

    def df(self, term: bytes):
        return lib().orc_df(self._ix, term, len(term))

    def vocab(self):
        """{term: df} for the shard."""
        V = self.num_terms
        buf = C.create_string_buffer(V * 257 + 16)
        df = np.zeros(max(V, 1), np.uint32)
        n = lib().orc_vocab(self._ix, buf, len(buf), _p(df, C.c_uint32), V)
        if n < 0:
            raise RuntimeError("orc_vocab rc=%d" % n)
        terms = buf.raw.split(b"\0")[:n]
        return dict(zip(terms, df[:n].tolist()))

    def set_global_stats(self, doc_count, sum_ttf, df_by_term):
        lib().orc_set_global_stats(self._ix, 0, 0)
        lib().orc_set_global_stats(self._ix, doc_count, sum_ttf)
        for t, v in df_by_term.items():
            lib().orc_set_global_df(self._ix, t, len(t), v)

    def search(self, q: bytes, k=0):
        """[(doc, score)] in (score desc, doc asc) order; k == 0 -> all hits."""
        cap = max(self.num_docs, 1)
        docs = np.zeros(cap, np.uint32)
        scores = np.zeros(cap, np.float32)
        n = C.c_uint64(0)
        rc = lib().orc_search(self._ix, q, len(q), k, _p(docs, C.c_uint32), _p(scores, C.c_float),
                              cap, C.byref(n))
        if rc == E_UNSUPPORTED:
            raise ValueError("query rejected (unsupported)")
        if rc == E_SYNTAX:
            raise QuerySyntaxError("query does not parse")
        if rc != OK:
            raise RuntimeError("orc_search rc=%d" % rc)
        return list(zip(docs[:n.value].tolist(), scores[:n.value].tolist()))


def idf(df, doc_count):
    return lib().orc_idf(df, doc_count)


def avgdl(sum_ttf, doc_count):
    return lib().orc_avgdl(sum_ttf, doc_count)


def norm_cache(k1, b, avg):
    out = np.zeros(256, np.float32)
    lib().orc_norm_cache(k1, b, avg, _p(out, C.c_float))
    return out


def bm25(weight, tf, norm_inverse):
    return lib().orc_bm25(weight, tf, norm_inverse)


def leader_merge(responses):
    """responses: list (worker order) of lists of (name bytes, double score).
    Returns [(name, summed score)] ordered by name (Leader.java:73-88)."""
    flat = [x for r in responses for x in r]
    n = len(flat)
    if n == 0:
        return []
    names = b"".join(nm for nm, _ in flat)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(nm) for nm, _ in flat])
    sc = np.array([s for _, s in flat], np.float64)
    first = np.zeros(n, np.uint64)
    sums = np.zeros(n, np.float64)
    m = lib().orc_leader_merge(names, _p(offs, C.c_uint64), n, _p(sc, C.c_double),
                               _p(first, C.c_uint64), _p(sums, C.c_double))
    return [(flat[int(first[i])][0], float(sums[i])) for i in range(m)]


def bulk_build(text, offsets, n_threads):
    """CPU baseline (bench.py only): n_threads C threads, each indexing its own
    contiguous share of the corpus (uint8 text, uint64 offsets[n + 1]) into
    its own index; no Python in the timed region.  -> (seconds, sum_ttf)."""
    import numpy as np
    text = np.ascontiguousarray(text, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    sec, ttf = C.c_double(), C.c_uint64()
    rc = lib().orc_bulk_build(C.c_void_p(text.ctypes.data), _p(offsets, C.c_uint64), len(offsets) - 1,
                              n_threads, C.byref(sec), C.byref(ttf))
    if rc != 0:
        raise RuntimeError("orc_bulk_build failed: %d" % rc)
    return sec.value, ttf.value
