#!/usr/bin/env python3
"""cfg-4 batch (10k 3-term queries, top-k) over the cfg-2 index: the query-unit
path (k_score_units) against the wave-per-pair path (TFIDF_NO_UNITS), device
time best of 5, and the two result sets compared."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tf-idf-distributed-system_amd"))

from tfidf_amd import synth  # noqa: E402
from tfidf_amd.engine import ShardIndex  # noqa: E402


def timed(g, bq, k, reps=5):
    best, res = None, None
    for _ in range(reps):
        res = g.search_batch(bq, k)
        sc, tot = g.last_search_ms()
        best = (sc, tot) if best is None or tot < best[1] else best
    return best, res


def main():
    n = int(os.environ.get("DOCS", "1000000"))
    dc = synth.DeviceCorpus(n)
    g = ShardIndex()
    g.add_documents_device(dc.d_text, dc.d_offsets, dc.n_docs, dc.total_bytes)
    g.commit()
    bq = synth.queries(int(os.environ.get("NQ", "10000")))
    g.search_batch(bq[:100], 10)
    if os.environ.get("LIGHTS"):                          # sweep of the light-query threshold (postings/block)
        for lt in os.environ["LIGHTS"].split(","):
            os.environ["TFIDF_WUNIT_LIGHT"] = lt
            (sc, tot), _ = timed(g, bq, 10)
            print("light<=%s: scoring %.3f total %.3f ms" % (lt, sc, tot), flush=True)
        os.environ.pop("TFIDF_WUNIT_LIGHT")
    if os.environ.get("WGS"):                             # sweep: workgroup units per CU next to the wave units
        for v in os.environ["WGS"].split(","):
            os.environ["TFIDF_UNIT_WG_PER_CU"] = v
            (sc, tot), _ = timed(g, bq, 10)
            print("wg/cu=%s: scoring %.3f total %.3f ms" % (v, sc, tot), flush=True)
        os.environ.pop("TFIDF_UNIT_WG_PER_CU")
    if os.environ.get("ONLY_UNITS"):                     # profiling: the unit path alone, k = 10
        for _ in range(2):
            g.search_batch(bq, 10)
        print("units k=10 ms", g.last_search_ms(), flush=True)
        g.close()
        dc.free()
        return
    for k in (10, 64):
        os.environ.pop("TFIDF_NO_UNITS", None)
        (usc, utot), (d1, s1, c1) = timed(g, bq, k)
        os.environ["TFIDF_NO_UNITS"] = "1"
        (psc, ptot), (d2, s2, c2) = timed(g, bq, k)
        os.environ.pop("TFIDF_NO_UNITS", None)
        same = bool(np.array_equal(c1, c2))
        if same:
            for i in range(len(bq)):
                c = c1[i]
                if not (np.array_equal(d1[i, :c], d2[i, :c]) and
                        np.array_equal(s1[i, :c].view(np.int32), s2[i, :c].view(np.int32))):
                    same = False
                    print("mismatch query", i, bq[i])
                    break
        print("k=%d units: scoring %.3f ms total %.3f ms | pairs: scoring %.3f total %.3f | identical %s | %s"
              % (k, usc, utot, psc, ptot, same, {x: g.stats()[x] for x in ("unit_batches", "unit_count")}),
              flush=True)
    g.close()
    dc.free()


if __name__ == "__main__":
    main()
