#!/usr/bin/env python3
"""A/B timing of the cfg-2 index build (1 M docs) between builds of
libtfidf.so (and TFIDF_TOKENIZER settings).  Usage: ab_build.py LIB[:ENV=VAL] ..."""
import ctypes as C
import os
import subprocess
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
    args = dict(a.split("=") for a in os.environ.get("AB_CORPUS", "").split(",") if a)
    n = int(args.get("docs", 1_000_000))
    dc = synth.DeviceCorpus(n, V=int(args.get("V", 100_000)), len_min=int(args.get("lmin", 400)),
                            len_max=int(args.get("lmax", 600)))
    g = ShardIndex(vocab_capacity_log2=int(args.get("cap", 18)))
    g.add_documents_device(dc.d_text, dc.d_offsets, dc.n_docs, dc.total_bytes)
    best = None
    for _ in range(5):
        g.commit()
        t = g.commit_timing()
        if best is None or t["ms_total"] < best["ms_total"]:
            best = t
    st = g.stats()
    print("%-28s %-22s total %.3f tok %.3f long %.3f df %.3f scan %.3f scat %.3f | terms %d nnz %d ttf %d long %d" % (
        os.path.basename(path), os.environ.get("TFIDF_TOKENIZER", ""), best["ms_total"], best["ms_tokenize"],
        best["ms_long"], best["ms_df"], best["ms_blockscan"] + best["ms_colscan"], best["ms_scatter"],
        st["num_terms"], st["nnz"], st["sum_ttf"], st["long_docs"]), flush=True)
    g.close()
    dc.free()


if __name__ == "__main__":
    if len(sys.argv) == 2 and ":" not in sys.argv[1]:
        run(sys.argv[1])
    else:
        for a in sys.argv[1:]:
            path, _, envs = a.partition(":")
            env = dict(os.environ)
            for kv in envs.split(";") if envs else []:
                k, v = kv.split("=")
                env[k] = v
            subprocess.check_call([sys.executable, __file__, path], env=env)
