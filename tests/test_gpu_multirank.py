"""The multi-GPU orchestration over the REAL engine: world size 2 and 3,
every rank a process with its own HipShardAdapter / ShardIndex on cuda:0,
collectives over gloo (RCCL needs one GPU per rank; the 8-GPU RCCL run is the
driver's).  Same rank body and checks as test_distributed_gloo.py
(tests/multirank.py): GLOBAL term-ownership and canonical statistics, top-k /
all-hits / batched merges with device merge keys, and SHARD mode's
Leader-style merge by name — all against the CPU oracle.
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
