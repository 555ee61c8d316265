#!/usr/bin/env python3
"""Single top-10 query latency on the cfg-2 index: p50/p99 of the C call
alone (ctypes, preallocated arrays) and of engine.search_arrays."""
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
    qs = synth.queries(400)
    lib = L.load()
    docs = np.zeros(10, np.uint32)
    scores = np.zeros(10, np.float32)
    n = C.c_uint64()
    pd, ps = L.ptr(docs, C.c_uint32), L.ptr(scores, C.c_float)
    for label, env in (("timing events", None), ("no timing events", "1")):
        if env:
            os.environ["TFIDF_NO_QTIMING"] = env
        else:
            os.environ.pop("TFIDF_NO_QTIMING", None)
        for q in qs[:20]:
            lib.tfidf_search(g._h, q, len(q), 10, pd, ps, 10, C.byref(n))
        lat = []
        for q in qs:
            t0 = time.perf_counter()
            lib.tfidf_search(g._h, q, len(q), 10, pd, ps, 10, C.byref(n))
            lat.append(time.perf_counter() - t0)
        lat2 = []
        for q in qs:
            t0 = time.perf_counter()
            g.search_arrays(q, 10)
            lat2.append(time.perf_counter() - t0)
        print("%-18s C call p50 %.1f us p99 %.1f | search_arrays p50 %.1f us" % (
            label, np.percentile(lat, 50) * 1e6, np.percentile(lat, 99) * 1e6, np.percentile(lat2, 50) * 1e6), flush=True)
    g.close()
    dc.free()


if __name__ == "__main__":
    main()
