#!/usr/bin/env python3
"""Stage times of distributed.global_commit (term-ownership GLOBAL statistics)
on the cfg-2 shard, under torch.distributed.run (nccl = RCCL; one rank on a
1-GPU box).  Each stage is closed by torch.cuda.synchronize()."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tf-idf-distributed-system_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tfidf_amd import STATS_GLOBAL, synth  # noqa: E402
from tfidf_amd import distributed as D  # noqa: E402
from tfidf_amd.engine import ShardIndex  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    corpus = synth.DeviceCorpus(1_000_000, device=local)
    idx = ShardIndex(device=local, stats_mode=STATS_GLOBAL)
    idx.add_documents_device(corpus.d_text, corpus.d_offsets, corpus.n_docs, corpus.total_bytes)
    idx.commit()
    ad = D.HipShardAdapter(idx, dev)
    D.global_commit(ad)
    ws, me = dist.get_world_size(), dist.get_rank()
    for rep in range(4):
        if os.environ.get("COMMIT"):                  # as bench.py's step: a fresh commit first
            idx.commit()
        T = []
        torch.cuda.synchronize()
        T.append(time.perf_counter())
        dc, ttf, _ = ad.local_stats()
        seed = ad.hash_seed()
        T.append(time.perf_counter())
        rec, cnt = ad.vocab_partition(ws)
        torch.cuda.synchronize()
        T.append(time.perf_counter())
        meta = torch.cat([cnt.to(torch.int64), torch.tensor([dc, ttf, seed], dtype=torch.int64, device=dev)])
        M = D._all_gather(meta, None).cpu().tolist()
        T.append(time.perf_counter())
        send = [int(x) for x in M[me][:ws]]
        recv = [int(M[r][me]) for r in range(ws)]
        got = torch.empty((sum(recv), 3), dtype=torch.int64, device=dev)
        D._a2a(got, rec.contiguous(), recv, send, None)
        torch.cuda.synchronize()
        T.append(time.perf_counter())
        ans, nu = ad.vocab_reduce(got)
        torch.cuda.synchronize()
        T.append(time.perf_counter())
        back = torch.empty(sum(send), dtype=torch.int32, device=dev)
        D._a2a(back, ans.contiguous(), send, recv, None)
        torch.cuda.synchronize()
        T.append(time.perf_counter())
        ad.import_global_df(back, dc, ttf)
        torch.cuda.synchronize()
        T.append(time.perf_counter())
        if os.environ.get("COMMIT"):
            idx.commit()
        t0 = time.perf_counter()
        D.global_commit(ad)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        names = ["stats", "partition", "meta_gather", "a2a_out", "reduce", "a2a_back", "import"]
        print("rep %d: " % rep + "  ".join("%s %.3f" % (n, (T[i + 1] - T[i]) * 1e3) for i, n in enumerate(names)),
              "| staged total %.3f ms | global_commit %.3f ms" % ((T[-1] - T[0]) * 1e3, (t1 - t0) * 1e3), flush=True)
    idx.close()
    corpus.free()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
