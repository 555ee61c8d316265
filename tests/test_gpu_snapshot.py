"""Snapshot-isolated concurrent search (include/tfidf.h "Threading"; the
reference opens a DirectoryReader on the last commit per request,
Worker.java:223, while an upload's synchronized add + commit runs beside it,
:136-139).

A writer thread re-commits the index over and over, toggling 300 documents
between two texts by replace-by-key; 16 threads search meanwhile — readers
(top-k and all hits, hits mapped to keys through the same reader), plain
tfidf_search top-k and batched top-k.  Every answer must equal the oracle of
one of the two corpus states (a batch: one state for all of its queries), and
both states must be seen.  Compared by (key, score): replace-by-key moves the
replaced documents to the end, so doc ids differ between commits of one state.
"""
import threading
import time

import numpy as np
import pytest

from oracle import oracle as O
from tfidf_amd import synth
from tfidf_amd.engine import ShardIndex

pytestmark = pytest.mark.gpu

N, R, K = 3000, 300, 10


def states():
    base = synth.corpus(N, V=5000, len_min=30, len_max=120)
    alt = synth.corpus(R, V=5000, len_min=30, len_max=120, seed=777)
    keys = [b"d%05d.txt" % i for i in range(N)]
    return keys, base, alt


QUERIES = synth.queries(12, lo=1, hi=800) + [b"aaaa", b"aaab aaac"]


def oracle_maps(keys, texts):
    o = O.OracleIndex()
    for k, t in zip(keys, texts):
        o.add_doc(k, t)
    o.commit()
    out = []
    for q in QUERIES:
        hits = o.search(q, 0)
        out.append({o.doc_key(d): np.float32(s) for d, s in hits})
    o.close()
    return out


def topk_scores(m, k):
    return sorted(m.values(), reverse=True)[:k]


def test_searches_see_one_committed_state_while_the_writer_commits():
    keys, base, alt = states()
    state_b = alt + base[R:]
    want = [oracle_maps(keys, base), oracle_maps(keys, state_b)]
    idx = ShardIndex(device=0)
    idx.add_documents(base, keys)
    idx.commit()
    stop = threading.Event()
    errors, seen = [], [[0, 0] for _ in range(16)]
    commits = [0]

    def writer():
        try:
            flip = 0
            while commits[0] < 16:
                flip ^= 1
                idx.add_documents(alt if flip else base[:R], keys[:R])
                idx.commit()
                commits[0] += 1
        except Exception as e:          # noqa: BLE001
            errors.append(("writer", repr(e)))
        finally:
            stop.set()

    def which(got_map, qi):
        return [s for s in (0, 1) if got_map == want[s][qi]]

    def check_topk(scores, qi):
        return [s for s in (0, 1) if [np.float32(x) for x in scores] == topk_scores(want[s][qi], K)]

    def reader_thread(t):
        i = 0
        while not stop.is_set() or i < 4:
            qi = (t + i) % len(QUERIES)
            with idx.reader() as rd:
                hits = rd.search(QUERIES[qi], 0)
                got = {rd.doc_key(d): np.float32(s) for d, s in hits}
                top = rd.search(QUERIES[qi], K)
                topm = [(rd.doc_key(d), np.float32(s)) for d, s in top]
            st = which(got, qi)
            if not st:
                errors.append(("reader all hits", t, qi))
                return
            if check_topk([s for _, s in topm], qi) != st or any(want[st[0]][qi].get(k) != s for k, s in topm):
                errors.append(("reader top-k", t, qi))
                return
            seen[t][st[0]] += 1
            i += 1

    def plain_thread(t):
        i = 0
        while not stop.is_set() or i < 4:
            qi = (t + i) % len(QUERIES)
            st = check_topk([s for _, s in idx.search(QUERIES[qi], K)], qi)
            if not st:
                errors.append(("search top-k", t, qi))
                return
            seen[t][st[0]] += 1
            i += 1

    def batch_thread(t):
        i = 0
        while not stop.is_set() or i < 2:
            d, sc, cnt = idx.search_batch(QUERIES, K)
            ok = [set(check_topk(sc[qi, :cnt[qi]].tolist(), qi)) for qi in range(len(QUERIES))]
            common = set.intersection(*ok)
            if not common:
                errors.append(("batch", t, [sorted(x) for x in ok]))
                return
            seen[t][min(common)] += 1
            i += 1

    fns = [reader_thread] * 8 + [plain_thread] * 4 + [batch_thread] * 4
    th = [threading.Thread(target=f, args=(i,), daemon=True) for i, f in enumerate(fns)]
    w = threading.Thread(target=writer, daemon=True)
    t0 = time.time()
    for x in th:
        x.start()
    w.start()
    w.join(120)
    for x in th:
        x.join(120)
    assert not w.is_alive() and not any(x.is_alive() for x in th), "a thread did not finish"
    assert not errors, errors[:5]
    assert commits[0] == 16
    tot = np.array(seen).sum(axis=0)
    print("searches per state", tot.tolist(), "in %.2f s" % (time.time() - t0))
    assert tot.sum() >= 16 * 2
    # the last commit (an even number of flips) published state 0 again
    with idx.reader() as rd:
        assert {rd.doc_key(d): np.float32(s) for d, s in rd.search(QUERIES[0], 0)} == want[0][0]
    idx.close()


def test_reader_keeps_its_snapshot_across_commits():
    keys, base, alt = states()
    idx = ShardIndex(device=0)
    idx.add_documents(base, keys)
    idx.commit()
    rd = idx.reader()
    g0 = rd.generation
    before = rd.search(QUERIES[0], 0)
    idx.add_documents(alt, keys[:R])
    idx.add_documents([b"zzzz extra document"], [b"new.txt"])
    idx.commit()
    assert idx.stats()["num_docs"] == N + 1
    assert rd.num_docs == N and rd.generation == g0
    assert rd.search(QUERIES[0], 0) == before                 # the pinned snapshot
    blob, offs = rd.doc_keys()
    assert len(offs) == N + 1 and bytes(blob[:offs[1]]) == keys[0]
    with idx.reader() as r2:
        assert r2.generation == g0 + 1 and r2.num_docs == N + 1
        assert r2.doc_key(N) == b"new.txt"
    rd.close()
    # documents added after a commit stay invisible until the next commit
    idx.add_documents([b"qqqq"], [b"later.txt"])
    assert idx.stats()["num_docs"] == N + 1
    assert idx.search(b"qqqq", 0) == []
    idx.commit()
    assert len(idx.search(b"qqqq", 0)) == 1
    idx.close()
