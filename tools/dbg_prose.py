import os, sys, random
sys.path.insert(0, "tests"); sys.path.insert(0, "tf-idf-distributed-system_amd"); sys.path.insert(0, ".")
os.environ.setdefault("TFIDF_DEBUG", "1")
import torch  # noqa
import test_gpu_uni_wave as T
from test_gpu_unicode_sparse import build_pair
from tfidf_amd import synth
rng = random.Random(97)
texts = T.prose_edge_docs()
prose = [T.doc(rng, rng.randint(20, 500), rng.randint(1, 12), T.PROSE + T.WORDS + T.JOIN) for _ in range(900)]
declined = [T.doc(rng, rng.randint(20, 300), 2, T.PROSE) + " 中文".encode() for _ in range(100)]
texts += prose + declined
texts += synth.corpus(200, V=3000, len_min=50, len_max=400)
rng.shuffle(texts)
g, o = build_pair(texts)
bad = 0
for d in range(len(texts)):
    a, b = g.doc_terms(d), o.doc_terms(d)
    if a != b:
        bad += 1
        sa, sb = dict(a), dict(b)
        print("doc", d, "gpu-only", {k: v for k, v in sa.items() if sb.get(k) != v}, "oracle-only", {k: v for k, v in sb.items() if sa.get(k) != v})
        t = texts[d]
        for k in list({k for k in sa if sb.get(k) != sa[k]} | {k for k in sb if sa.get(k) != sb[k]})[:3]:
            kk = k if isinstance(k, bytes) else k.encode()
            i = t.lower().find(kk.split(b"\xe2")[0][:4]) if kk else -1
        print("   text:", t[:300])
        if bad > 5: break
print("mismatching docs", bad)
