#!/usr/bin/env python3
"""A/B timing of the cfg-4 batch (10k 3-term queries, top-10) over the cfg-2
index between two builds of libtfidf.so.  Usage: ab_batch.py LIB [LIB ...]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tf-idf-distributed-system_amd"))


def run(path):
    from tfidf_amd import _lib as L
    lib = C.CDLL(path)
    for name, (res, args) in L.SIGNATURES.items():
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
    L._lib = lib
    from tfidf_amd import synth
    from tfidf_amd.engine import ShardIndex
    dc = synth.DeviceCorpus(1_000_000)
    g = ShardIndex()
    g.add_documents_device(dc.d_text, dc.d_offsets, dc.n_docs, dc.total_bytes)
    g.commit()
    bq = synth.queries(10_000)
    g.search_batch(bq[:100], 10)
    out = []
    for k in (10, 100):
        best = None
        for _ in range(3):
            g.search_batch(bq, k)
            sc, tot = g.last_search_ms()
            best = tot if best is None else min(best, tot)
        out.append("k=%d %.2f ms" % (k, best))
    print(os.path.basename(path), *out, flush=True)
    g.close()
    dc.free()


if __name__ == "__main__":
    import subprocess
    if len(sys.argv) == 2:
        run(sys.argv[1])
    else:
        for p in sys.argv[1:]:
            subprocess.check_call([sys.executable, __file__, p])
