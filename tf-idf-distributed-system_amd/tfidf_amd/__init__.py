"""tfidf_amd — host layer of the MI355X-native TF-IDF/BM25 engine.

The compute runs in libtfidf.so (HIP kernels for gfx950, C ABI in
include/tfidf.h).  This package binds it with ctypes and mirrors the
reference's Worker/Leader interface (reference_api) plus the multi-GPU
orchestration (distributed).
"""
from ._lib import (STATS_GLOBAL, STATS_SHARD, TfidfError, UnsupportedInput, UnsupportedQuery, build,  # noqa: F401
                   load)
from .engine import ShardIndex, leader_merge, term_key  # noqa: F401
