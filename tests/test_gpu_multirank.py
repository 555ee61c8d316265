"""The node-level orchestration of libtfidf (tfidf_dist_*, process model (2):
one process per rank) over the REAL engine: world size 2 and 3, every rank a
process with its own ShardIndex on cuda:0, the library's collectives through a
callback communicator on a gloo group (RCCL needs one GPU per rank; the 8-GPU
RCCL run is the driver's).  GLOBAL term-ownership statistics, top-k /
all-hits / batched merges of device merge keys, and SHARD mode's Leader-style
merge by name — all against the CPU oracle (tests/multirank.py).
"""
import json

import pytest
import torch.multiprocessing as mp

import multirank as M

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 3])
def test_hip_adapter_multirank(tmp_path, world):
    out = str(tmp_path / "r.json")
    mp.spawn(M.run_rank, args=(world, M.free_port(), "hip", out), nprocs=world, join=True)
    M.check(json.load(open(out)), world)


def test_hip_hash_seed_agreement(tmp_path):
    """Shard 1 meets hash collisions (TFIDF_TEST_WEAK_HASH) and commits under
    seed attempt 1; shard 0 re-commits under it and GLOBAL statistics and
    rankings equal the single-index oracle."""
    out = str(tmp_path / "s.json")
    mp.spawn(M.run_rank_seed, args=(2, M.free_port(), "hip", out), nprocs=2, join=True)
    res = M.check_seed(out, 2)
    assert [r["before"] for r in res] == [0, 1]
    assert [r["after"] for r in res] == [1, 1]
