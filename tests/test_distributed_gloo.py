"""World-size-2 (and 3) CPU rehearsal of the multi-GPU orchestration in
tfidf_amd/distributed.py over the gloo backend.  The per-rank engine is the
CPU oracle behind the same adapter interface HipShardAdapter implements
(tests/multirank.py); the orchestration code under test is the production
code: GLOBAL statistics by term ownership and by the canonical union, top-k,
all-hits and batched merges, and SHARD mode (every worker's hits summed by
document name in rank order, ordered by name — Leader.java:39-92).

GLOBAL mode over G shards must equal the single-index (1-worker) result;
SHARD mode must equal per-worker oracles + the oracle's Leader merge.
(test_gpu_multirank.py runs the same rank body over the HIP engine.)
"""
import json

import pytest
import torch.multiprocessing as mp

import multirank as M


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_modes_equal_oracle(tmp_path, world):
    out = str(tmp_path / "r.json")
    mp.spawn(M.run_rank, args=(world, M.free_port(), "oracle", out), nprocs=world, join=True)
    M.check(json.load(open(out)), world)


def test_hash_seed_agreement(tmp_path):
    """Shards that hashed with different seeds agree on the highest: the others
    re-commit under it (and agree again when that seed collides there)."""
    out = str(tmp_path / "s.json")
    mp.spawn(M.run_rank_seed, args=(3, M.free_port(), "oracle", out), nprocs=3, join=True)
    res = M.check_seed(out, 3)
    assert [r["before"] for r in res] == [0, 1, 0]
    assert [r["after"] for r in res] == [2, 2, 2]
    assert [r["recommits"] for r in res] == [[1, 2], [2], [1]]
