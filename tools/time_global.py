#!/usr/bin/env python3
"""Per-step cost of the GLOBAL-statistics exchange on one GPU, without the
collectives: vocabulary export, canonicalisation of a G-rank all-gather
result (G copies of this shard's vocabulary, i.e. the worst case where every
rank holds the same terms), canonical DF import.  Usage: time_global.py [G...]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tf-idf-distributed-system_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from tfidf_amd import STATS_GLOBAL, synth  # noqa: E402
from tfidf_amd import distributed as D  # noqa: E402
from tfidf_amd.engine import ShardIndex  # noqa: E402


def main():
    gs = [int(x) for x in sys.argv[1:]] or [2, 8]
    dev = torch.device("cuda", 0)
    corpus = synth.DeviceCorpus(1_000_000, doc_base=0)
    idx = ShardIndex(stats_mode=STATS_GLOBAL)
    idx.add_documents_device(corpus.d_text, corpus.d_offsets, corpus.n_docs, corpus.total_bytes)
    idx.commit()
    ad = D.HipShardAdapter(idx, dev)
    for G in gs:
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            keys, df = ad.export_vocab()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            all_keys = torch.cat([keys] * G, 0).contiguous()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            dfc = ad.canonicalize(all_keys)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            dc, ttf, _ = ad.local_stats()
            ad.import_global(dfc * G, dc * G, ttf * G)
            torch.cuda.synchronize()
            t4 = time.perf_counter()
        print("canonical G=%d vocab=%d  export %.2f ms  concat %.2f ms  canonicalize %.2f ms  import %.2f ms  "
              "total %.2f ms" % (G, keys.shape[0], (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3,
                                 (t4 - t3) * 1e3, (t4 - t0) * 1e3), flush=True)
        # term ownership: each owner receives ~vocab records in total when every rank holds every term
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rec, counts = ad.vocab_partition(G)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ans, nu = ad.vocab_reduce(rec)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            dc, ttf, _ = ad.local_stats()
            ad.import_global_df(ans, dc, ttf)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
        print("ownership G=%d records=%d  partition %.2f ms  reduce %.2f ms  import %.2f ms  total %.2f ms"
              % (G, rec.shape[0], (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t3 - t0) * 1e3), flush=True)
    corpus.free()
    idx.close()


if __name__ == "__main__":
    main()
