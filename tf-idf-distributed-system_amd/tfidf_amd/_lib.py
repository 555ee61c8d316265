"""ctypes binding of libtfidf.so (include/tfidf.h).

The library is built in-tree (``make -C tf-idf-distributed-system_amd``) and
loaded from ``tf-idf-distributed-system_amd/lib/libtfidf.so``.  There is no
fallback: if the HIP library is missing, every engine call raises.
"""
import ctypes as C
import os
import subprocess

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libtfidf.so")

OK = 0
E_INVALID_ARG = 1
E_HIP = 2
E_OOM = 3
E_UNSUPPORTED_INPUT = 4
E_UNSUPPORTED_QUERY = 5
E_CAPACITY = 6
E_STATE = 7
E_BUFFER = 8
E_NO_DEVICE = 9
E_QUERY_SYNTAX = 10

STATS_SHARD = 0
STATS_GLOBAL = 1

OWN_STREAM = C.c_void_p(-1 & ((1 << 64) - 1))   # TFIDF_OWN_STREAM

INVERSION_AUTO = 0
INVERSION_BLOCK = 1
INVERSION_TERM = 2


class Config(C.Structure):
    _fields_ = [("k1", C.c_float), ("b", C.c_float), ("stats_mode", C.c_int32), ("device", C.c_int32),
                ("vocab_capacity_log2", C.c_uint32), ("max_token_len", C.c_uint32), ("inversion", C.c_int32)]


class IndexStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("num_docs", "doc_count", "sum_ttf", "num_terms", "nnz",
                                          "device_bytes", "long_docs", "text_bytes", "term_major",
                                          "pack_docs", "pack_retried", "unicode_docs", "long_chunked",
                                          "malformed_docs", "hash_seed", "hash_rebuilds",
                                          "coalesced_batches", "coalesced_queries", "unit_batches", "unit_count", "fused_queries",
                                          "unicode_wave_docs")]


class CommitTiming(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("ms_total", "ms_tokenize", "ms_long", "ms_df", "ms_blockscan",
                                         "ms_colscan", "ms_scatter")] + \
               [(n, C.c_uint64) for n in ("text_bytes", "num_docs", "nnz")]


class TfidfError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("libtfidf error %d: %s" % (code, msg))
        self.code = code


class UnsupportedQuery(TfidfError):
    pass


class UnsupportedInput(TfidfError):
    pass


class QuerySyntaxError(TfidfError):
    """QueryParser ParseException / TooManyClauses: Worker.processDocuments answers []."""


VP = C.c_void_p
U8P = C.POINTER(C.c_uint8)
U32P = C.POINTER(C.c_uint32)
U64P = C.POINTER(C.c_uint64)
F32P = C.POINTER(C.c_float)
F64P = C.POINTER(C.c_double)

SIGNATURES = {
    "tfidf_version": (C.c_char_p, []),
    "tfidf_last_error": (C.c_char_p, []),
    "tfidf_config_init": (C.c_int, [C.POINTER(Config)]),
    "tfidf_create": (C.c_int, [C.POINTER(Config), C.POINTER(VP)]),
    "tfidf_destroy": (C.c_int, [VP]),
    "tfidf_add_docs": (C.c_int, [VP, VP, U64P, C.c_uint64, C.c_char_p, U64P]),
    "tfidf_clear": (C.c_int, [VP]),
    "tfidf_save": (C.c_int, [VP, C.c_char_p]),
    "tfidf_load": (C.c_int, [VP, C.c_char_p]),
    "tfidf_add_docs_device": (C.c_int, [VP, VP, VP, C.c_uint64, C.c_uint64]),
    "tfidf_commit": (C.c_int, [VP]),
    "tfidf_set_hash_attempt": (C.c_int, [VP, C.c_uint32]),
    "tfidf_get_commit_timing": (C.c_int, [VP, C.POINTER(CommitTiming)]),
    "tfidf_stats": (C.c_int, [VP, C.POINTER(IndexStats)]),
    "tfidf_search": (C.c_int, [VP, C.c_char_p, C.c_uint64, C.c_uint32, U32P, F32P, C.c_uint64, U64P]),
    "tfidf_search_coalesced": (C.c_int, [VP, C.c_char_p, C.c_uint64, C.c_uint32, U32P, F32P, C.c_uint64, U64P,
                                         C.c_uint32]),
    "tfidf_search_batch": (C.c_int, [VP, C.c_char_p, U64P, C.c_uint32, C.c_uint32, U32P, F32P, U32P]),
    "tfidf_last_search_ms": (C.c_int, [VP, F32P, F32P]),
    "tfidf_set_query_timing": (C.c_int, [VP, C.c_int]),
    "tfidf_search_batch_keys_device": (C.c_int, [VP, C.c_char_p, U64P, C.c_uint32, C.c_uint32, C.c_uint64, VP]),
    "tfidf_search_all_keys_device": (C.c_int, [VP, C.c_char_p, C.c_uint64, C.c_uint64, VP, C.c_uint64, U64P]),
    "tfidf_set_stream": (C.c_int, [VP, VP]),
    "tfidf_doc_keys": (C.c_int, [VP, C.c_char_p, C.c_uint64, U64P, U64P]),
    "tfidf_sort_names": (C.c_int, [C.c_char_p, U64P, C.c_uint64, U64P]),
    "tfidf_doc_key": (C.c_int, [VP, C.c_uint64, C.c_char_p, C.c_uint64, U64P]),
    "tfidf_doc_len": (C.c_int, [VP, C.c_uint64, U32P, U8P]),
    "tfidf_malformed_docs": (C.c_int, [VP, U64P, C.c_uint64, U64P]),
    "tfidf_doc_terms": (C.c_int, [VP, C.c_uint64, C.c_char_p, C.c_uint64, U32P, C.c_uint64, U64P]),
    "tfidf_term_df": (C.c_int, [VP, C.c_char_p, C.c_uint64, U64P, U64P]),
    "tfidf_vocab_size": (C.c_int, [VP, U64P]),
    "tfidf_vocab_export": (C.c_int, [VP, U64P, U32P, U32P, C.c_uint64, U64P]),
    "tfidf_vocab_export_device": (C.c_int, [VP, VP, VP, C.c_uint64, U64P]),
    "tfidf_vocab_canonicalize_device": (C.c_int, [VP, VP, C.c_uint64, VP, C.c_uint64, U64P]),
    "tfidf_set_global_stats_device": (C.c_int, [VP, VP, C.c_uint64, C.c_uint64, C.c_uint64]),
    "tfidf_vocab_partition_device": (C.c_int, [VP, C.c_uint32, VP, C.c_uint64, VP, U64P]),
    "tfidf_vocab_reduce_device": (C.c_int, [VP, VP, C.c_uint64, VP, VP]),
    "tfidf_set_global_df_device": (C.c_int, [VP, VP, C.c_uint64, C.c_uint64, C.c_uint64]),
    "tfidf_set_global_stats": (C.c_int, [VP, U64P, U64P, C.c_uint64, C.c_uint64, C.c_uint64]),
    "tfidf_clear_global_stats": (C.c_int, [VP]),
    "tfidf_term_key": (C.c_int, [C.c_char_p, C.c_uint64, U64P, U64P]),
    "tfidf_analyze": (C.c_int, [C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64, U64P, U64P]),
    "tfidf_leader_merge": (C.c_int, [C.c_char_p, U64P, C.c_uint64, F64P, U64P, F64P, U64P]),
    "tfidf_synth_corpus": (C.c_int, [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, F64P, C.c_uint32, C.c_uint32,
                                     C.c_uint32, C.POINTER(VP), C.POINTER(VP), U64P]),
    # node level (csrc/tfidf_dist.hip)
    "tfidf_comm_create": (C.c_int, [C.c_int32, C.c_int32, VP, C.POINTER(VP)]),
    "tfidf_rccl_unique_id": (C.c_int, [VP]),
    "tfidf_comm_init_rccl": (C.c_int, [VP, C.c_int32, C.c_int32, C.c_int32, C.POINTER(VP)]),
    "tfidf_comm_create_inproc": (C.c_int, [C.c_int32, C.POINTER(VP)]),
    "tfidf_comm_destroy": (C.c_int, [VP]),
    "tfidf_comm_info": (C.c_int, [VP, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "tfidf_comm_selftest": (C.c_int, [VP]),
    "tfidf_dist_global_commit": (C.c_int, [VP, VP, U64P, U64P, U64P]),
    "tfidf_dist_search": (C.c_int, [VP, VP, C.c_uint64, C.c_char_p, C.c_uint64, C.c_uint32, U64P, F32P, C.c_uint64,
                                    U64P]),
    "tfidf_dist_search_batch": (C.c_int, [VP, VP, C.c_uint64, C.c_char_p, U64P, C.c_uint32, C.c_uint32, U64P, F32P,
                                          U32P]),
    "tfidf_dist_shard_commit": (C.c_int, [VP, VP, U64P]),
    "tfidf_dist_shard_search": (C.c_int, [VP, VP, C.c_char_p, C.c_uint64, U64P, U64P]),
    "tfidf_dist_last_hits": (C.c_int, [VP, U64P, F32P, C.c_uint64, U64P]),
    "tfidf_dist_last_failed": (C.c_int, [VP, U64P]),
    "tfidf_reader_open": (C.c_int, [VP, C.POINTER(VP)]),
    "tfidf_reader_close": (C.c_int, [VP]),
    "tfidf_reader_info": (C.c_int, [VP, U64P, U64P]),
    "tfidf_reader_search": (C.c_int, [VP, C.c_char_p, C.c_uint64, C.c_uint32, U32P, F32P, C.c_uint64, U64P]),
    "tfidf_reader_doc_key": (C.c_int, [VP, C.c_uint64, C.c_char_p, C.c_uint64, U64P]),
    "tfidf_reader_doc_keys": (C.c_int, [VP, C.c_char_p, C.c_uint64, U64P, U64P]),
    "tfidf_dist_last_names": (C.c_int, [VP, C.c_char_p, C.c_uint64, U64P, F64P, C.c_uint64, U64P, U64P]),
    "tfidf_node_create": (C.c_int, [VP, C.c_uint64, C.POINTER(VP)]),
    "tfidf_node_create_devices": (C.c_int, [VP, C.POINTER(C.c_int32), C.c_uint32, C.c_uint32, C.POINTER(VP)]),
    "tfidf_node_destroy": (C.c_int, [VP]),
    "tfidf_node_shard": (C.c_int, [VP, C.c_uint32, C.POINTER(VP), U32P]),
    "tfidf_node_add_docs": (C.c_int, [VP, C.c_int32, C.c_char_p, U64P, C.c_uint64, C.c_char_p, U64P]),
    "tfidf_node_commit": (C.c_int, [VP]),
    "tfidf_node_search": (C.c_int, [VP, C.c_char_p, C.c_uint64, C.c_uint32, U64P, F32P, C.c_uint64, U64P]),
    "tfidf_node_search_batch": (C.c_int, [VP, C.c_char_p, U64P, C.c_uint32, C.c_uint32, U64P, F32P, U32P]),
    "tfidf_node_search_names": (C.c_int, [VP, C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64, U64P, F64P,
                                          C.c_uint64, U64P, U64P]),
    "tfidf_node_doc_key": (C.c_int, [VP, C.c_uint64, C.c_char_p, C.c_uint64, U64P]),
    "tfidf_node_last_failed": (C.c_int, [VP, U64P]),
    "tfidf_node_stats_get": (C.c_int, [VP, VP]),
    "tfidf_device_free": (C.c_int, [C.c_int, VP]),
    "tfidf_device_copy": (C.c_int, [C.c_int, VP, VP, C.c_uint64, C.c_int]),
}

_lib = None


def build(jobs=8):
    subprocess.check_call(["make", "-s", "-j%d" % jobs, "-C", PKG_ROOT])


def load():
    """Load libtfidf.so.  Raises if the HIP library is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libtfidf.so not built at %s (run __graft_entry__.build())" % LIB_PATH)
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def check(rc):
    if rc == OK:
        return
    msg = load().tfidf_last_error().decode(errors="replace")
    if rc == E_UNSUPPORTED_QUERY:
        raise UnsupportedQuery(rc, msg)
    if rc == E_UNSUPPORTED_INPUT:
        raise UnsupportedInput(rc, msg)
    if rc == E_QUERY_SYNTAX:
        raise QuerySyntaxError(rc, msg)
    raise TfidfError(rc, msg)


def ptr(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))
