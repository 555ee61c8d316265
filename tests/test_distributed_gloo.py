"""CPU tests of the node-level transports (csrc/tfidf_dist.hip, include/tfidf.h
"Node level"), no GPU needed: the orchestration's collectives go through a
tfidf_comm, and these check each transport end to end through the library.

* callback transport over a torch.distributed gloo group (world 2 and 3, one
  process per rank): the library calls the group's all_gather /
  all_to_all_single on host buffers through ctypes callbacks — the path the
  GPU multi-rank tests (ranks sharing one GPU) and a Java host with its own
  collectives take;
* in-process transport (world 1..5, one thread per rank): the transport
  tfidf_node uses for shards that share a device.

The orchestration itself over real shards (GLOBAL / SHARD results against the
oracle, hash-seed agreement) needs indices, i.e. a GPU: test_gpu_multirank.py,
test_gpu_node.py, test_gpu_fullsize_multirank.py.
"""
import threading

import pytest
import torch.multiprocessing as mp

import multirank as M


def _rank_selftest(rank, world, port):
    import os
    import torch.distributed as dist
    from tfidf_amd.distributed import Comm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = Comm.from_group(transport="callback")
    assert c.info() == (rank, world, "callback")
    for _ in range(3):
        c.selftest()
    c.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_callback_transport_gloo(world):
    mp.spawn(_rank_selftest, args=(world, M.free_port()), nprocs=world, join=True)


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_inproc_transport_threads(world):
    from tfidf_amd.distributed import Comm
    comms = Comm.inproc(world)
    errs = [None] * world

    def run(i):
        try:
            assert comms[i].info() == (i, world, "inproc")
            for _ in range(4):
                comms[i].selftest()
        except Exception as e:          # surfaced by the assert below
            errs[i] = e

    th = [threading.Thread(target=run, args=(i,)) for i in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th)
    assert errs == [None] * world
    for c in comms:
        c.close()


def test_comm_arguments_rejected():
    import ctypes as C
    from tfidf_amd import _lib as L
    from tfidf_amd.distributed import AG_FN, A2A_FN, Collectives
    lib = L.load()
    h = C.c_void_p()
    coll = Collectives(None, 0, AG_FN(lambda *a: 0), A2A_FN(lambda *a: 0))
    assert lib.tfidf_comm_create(2, 2, C.byref(coll), C.byref(h)) == L.E_INVALID_ARG     # rank >= world
    coll.memory = 7
    assert lib.tfidf_comm_create(0, 2, C.byref(coll), C.byref(h)) == L.E_INVALID_ARG     # unknown memory kind
    assert lib.tfidf_comm_create_inproc(0, (C.c_void_p * 1)()) == L.E_INVALID_ARG
