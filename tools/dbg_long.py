"""Diagnostic: which prose cfg-2 documents leave the wave paths (long_docs) and
whether the chunk path takes them (long_chunked); distinct terms per document
from the index itself (tfidf_doc_terms)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tf-idf-distributed-system_amd"))
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
scale = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
c = synth.DeviceCorpus(n, V=100_000, len_min=400, len_max=600, doc_base=0, device=0)
print("prose words", c.inject_prose(scale))
idx = ShardIndex(device=0, vocab_capacity_log2=19)
idx.add_documents_device(c.d_text, c.d_offsets, n, c.total_bytes)
idx.commit()
st = idx.stats()
print({k: st[k] for k in ("long_docs", "long_chunked", "unicode_docs", "unicode_wave_docs") if k in st})
nu = np.array([len(idx.doc_terms(d)) for d in range(n)])
print("distinct terms: max", nu.max(), "p99", np.percentile(nu, 99), "> 512:", int((nu > 512).sum()),
      "> 480:", int((nu > 480).sum()))
