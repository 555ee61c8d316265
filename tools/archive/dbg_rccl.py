"""Debug: RCCL world-1 transport vs the in-process one on the same shard."""
import ctypes as C
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tf-idf-distributed-system_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import torch  # noqa: F401,E402
import numpy as np  # noqa: E402
import multirank as M  # noqa: E402
from tfidf_amd import _lib as L  # noqa: E402
from tfidf_amd import distributed as D  # noqa: E402
from tfidf_amd.engine import ShardIndex  # noqa: E402

lib = L.load()
uid = (C.c_uint8 * 128)()
L.check(lib.tfidf_rccl_unique_id(uid))
h = C.c_void_p()
L.check(lib.tfidf_comm_init_rccl(uid, 0, 1, 0, C.byref(h)))
comm = D.Comm(h)
print("info", comm.info(), flush=True)
comm.selftest()
print("selftest ok", flush=True)
texts, names = M.corpus()
idx = ShardIndex(device=0)
idx.add_documents(texts, names)
idx.commit()
st = idx.stats()
k0, dl0, de0 = idx.vocab_export()
ad = D.DistShard(idx, comm, doc_base=0)
nv, dc, ttf = ad.global_commit(vocab_size=True)
print("local", st["num_terms"], st["doc_count"], st["sum_ttf"], "global", nv, dc, ttf, flush=True)
k1, dl1, de1 = idx.vocab_export()
bad = np.nonzero(de1 != dl1)[0]
print("df mismatches", len(bad), "of", len(dl1), (dl1[bad[:10]], de1[bad[:10]]) if len(bad) else "", flush=True)
q = M.QUERIES[0]
print("local", idx.search(q, 5))
print("dist ", ad.search(q, 5))
