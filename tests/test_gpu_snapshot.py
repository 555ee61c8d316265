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


LONG = b"supercalifragilisticexpialidocious"      # > 16 bytes: a hashed key, checked against its corpus spelling


def test_reader_keeps_its_snapshot_across_clear():
    """tfidf_clear restarts the staged corpus at offset 0: a reader pinned
    before it must keep reading its own corpus bytes (the spelling of hashed
    terms comes from the snapshot's text), not the new documents'."""
    idx = ShardIndex(device=0)
    texts = [b"%s alpha beta %d" % (LONG, i) for i in range(50)] + [b"gamma delta"] * 10
    idx.add_documents(texts, [b"a%03d" % i for i in range(60)])
    idx.commit()
    rd = idx.reader()
    before_long = rd.search(LONG, 0)
    before_alpha = rd.search(b"alpha", 5)
    assert len(before_long) == 50
    idx.clear()
    # different bytes over the same offsets (same lengths, other letters)
    idx.add_documents([b"x" * len(t) for t in texts], [b"b%03d" % i for i in range(60)])
    idx.commit()
    assert idx.search(LONG, 0) == []
    assert rd.search(LONG, 0) == before_long
    assert rd.search(b"alpha", 5) == before_alpha
    assert rd.doc_key(0) == b"a000"
    rd.close()
    idx.close()


def test_failed_searches_drain_before_their_snapshot_is_rebuilt(monkeypatch):
    """Every third scoring call fails after its kernels are queued
    (TFIDF_TEST_FAIL_SCORING, a test knob) while a writer re-commits states of
    different sizes, so the commit rebuilds (and regrows) the snapshots the
    failed searches held: no fault, and every search that succeeds equals the
    oracle of one committed state."""
    monkeypatch.setenv("TFIDF_TEST_FAIL_SCORING", "3")
    keys, base, _ = states()
    big = synth.corpus(R, V=5000, len_min=400, len_max=600, seed=778)
    state_b = big + base[R:]
    want = [oracle_maps(keys, base), oracle_maps(keys, state_b)]
    idx = ShardIndex(device=0)
    idx.add_documents(base, keys)
    idx.commit()
    stop = threading.Event()
    errors, fails, oks = [], [0], [0]

    def writer():
        try:
            for i in range(12):
                idx.add_documents(big if i % 2 == 0 else base[:R], keys[:R])
                idx.commit()
        except Exception as e:          # noqa: BLE001
            errors.append(("writer", repr(e)))
        finally:
            stop.set()

    def searcher(t):
        i = 0
        while not stop.is_set() or i < 3:
            qi = (t + i) % len(QUERIES)
            i += 1
            try:
                if t % 2:
                    hits = idx.search(QUERIES[qi], 0)              # all hits: through run_scoring
                    got = sorted((np.float32(s) for _, s in hits), reverse=True)
                    if not any(got == sorted(want[s][qi].values(), reverse=True) for s in (0, 1)):
                        errors.append(("all hits", t, qi))
                        return
                else:
                    d, sc, cnt = idx.search_batch(QUERIES, K)
                    ok = [set(s for s in (0, 1)
                              if [np.float32(x) for x in sc[q, :cnt[q]].tolist()] == topk_scores(want[s][q], K))
                          for q in range(len(QUERIES))]
                    if not set.intersection(*ok):
                        errors.append(("batch", t))
                        return
                oks[0] += 1
            except Exception as e:      # noqa: BLE001
                if "injected scoring failure" not in str(e):
                    errors.append(("search", t, repr(e)))
                    return
                fails[0] += 1

    th = [threading.Thread(target=searcher, args=(i,), daemon=True) for i in range(8)]
    w = threading.Thread(target=writer, daemon=True)
    for x in th:
        x.start()
    w.start()
    w.join(120)
    for x in th:
        x.join(120)
    assert not w.is_alive() and not any(x.is_alive() for x in th), "a thread did not finish"
    assert not errors, errors[:5]
    assert fails[0] > 0 and oks[0] > 0, (fails, oks)
    monkeypatch.delenv("TFIDF_TEST_FAIL_SCORING")
    idx.commit()
    with idx.reader() as rd:
        assert {rd.doc_key(d): np.float32(s) for d, s in rd.search(QUERIES[0], 0)} == want[0][0]
    idx.close()
