"""Per-step commit phases of the cfg-2 build (bench.py's workload), to see
whether a phase drifts over the steps: python tools/time_steps.py [steps] [prose]."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tf-idf-distributed-system_amd"))
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
prose = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
c = synth.DeviceCorpus(1_000_000, V=100_000, len_min=400, len_max=600, doc_base=0, device=0)
c.inject_prose(prose)
idx = ShardIndex(device=0, vocab_capacity_log2=19)
idx.add_documents_device(c.d_text, c.d_offsets, c.n_docs, c.total_bytes)
for i in range(steps):
    idx.commit()
    t = idx.commit_timing()
    st = idx.stats()
    print("step %2d tokenize %.3f long %.3f total %.3f uwave_docs %s rebuilds %s" % (i, t["ms_tokenize"], t["ms_long"],
          t["ms_total"], st.get("unicode_wave_docs"), st.get("hash_rebuilds")), flush=True)
