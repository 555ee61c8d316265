#!/usr/bin/env python3
"""Where a 10k-query batch's wall time goes: Python packing, the C call
(host preparation + upload + device + readback), the device time."""
import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tf-idf-distributed-system_amd"))

from tfidf_amd import _lib as L  # noqa: E402
from tfidf_amd import synth  # noqa: E402
from tfidf_amd.engine import ShardIndex  # noqa: E402


def main():
    dc = synth.DeviceCorpus(1_000_000)
    g = ShardIndex()
    g.add_documents_device(dc.d_text, dc.d_offsets, dc.n_docs, dc.total_bytes)
    g.commit()
    bq = synth.queries(10_000)
    g.search_batch(bq[:100], 10)
    k = 10
    for rep in range(4):
        t0 = time.perf_counter()
        nq = len(bq)
        offs = np.zeros(nq + 1, np.uint64)
        offs[1:] = np.cumsum([len(q) for q in bq], dtype=np.uint64)
        blob = b"".join(bq)
        docs = np.zeros((nq, k), np.uint32)
        scores = np.zeros((nq, k), np.float32)
        counts = np.zeros(nq, np.uint32)
        t1 = time.perf_counter()
        L.check(L.load().tfidf_search_batch(g._h, blob, L.ptr(offs, C.c_uint64), nq, k, L.ptr(docs, C.c_uint32),
                                            L.ptr(scores, C.c_float), L.ptr(counts, C.c_uint32)))
        t2 = time.perf_counter()
        sc, tot = g.last_search_ms()
        print("pack %.2f ms  C call %.2f ms  device %.2f ms  (host in C ~%.2f ms)  qps(wall) %.0f"
              % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, tot, (t2 - t1) * 1e3 - tot, nq / (t2 - t0)), flush=True)
    g.close()
    dc.free()


if __name__ == "__main__":
    main()
