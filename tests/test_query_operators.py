"""Query operator words (AND / OR / NOT) — the reference runs
QueryParser.parse(QueryParser.escape(q)) (Worker.java:225-227), and escape()
leaves the operator words alone, so Lucene 9.8.0 answers conjunctions and
exclusions.  CPU checks: the C oracle (oracle/tfidf_oracle.c) against an
independent pure-Python restatement of the same grammar, rewrite and scorer
shapes (numpy float32 arithmetic), on the reference's 8 sample documents and
on seeded random corpora.  Scores: parity unpinned (no Lucene artefact in the
image records one); the grammar cases below are the classic QueryParser's.
"""
import random

import numpy as np
import pytest

from oracle import oracle as O

F32 = np.float32


def py_parse(q: bytes):
    """-> list of [occur, [(token, count) ...]] after addClause, or None (ParseException)."""
    for w in ("\u3000".encode(), b"\t", b"\n", b"\r"):        # classic QueryParser _WHITESPACE
        q = q.replace(w, b" ")
    toks = [c for c in q.split(b" ") if c]
    kinds = [{b"AND": "AND", b"OR": "OR", b"NOT": "NOT"}.get(t, "TERM") for t in toks]
    clauses = []

    def add(conj, mods, chunk):
        if clauses and conj == "AND" and clauses[-1][0] != "MUST_NOT":
            clauses[-1][0] = "MUST"
        an = O.tokenize(chunk)
        if not an:
            return
        occ = "MUST_NOT" if mods == "NOT" else ("MUST" if conj == "AND" else "SHOULD")
        cnt = {}
        for t in an:
            cnt[t] = cnt.get(t, 0) + 1
        clauses.append([occ, list(cnt.items())])

    p, first = 0, True
    while first or p < len(kinds):
        conj = None
        if not first and kinds[p] in ("AND", "OR"):
            conj = kinds[p]
            p += 1
        mods = None
        if p < len(kinds) and kinds[p] == "NOT":
            mods = "NOT"
            p += 1
        if p >= len(kinds) or kinds[p] != "TERM":
            return None
        add(conj, mods, toks[p])
        p += 1
        first = False
    return clauses


def py_search(ix, q: bytes):
    """Rewrite + Boolean2ScorerSupplier shapes, float32 BM25Similarity."""
    clauses = py_parse(q)
    if clauses is None:
        return None
    N = ix.num_docs
    dc = ix.doc_count
    if dc == 0:
        return []
    avg = F32(ix.sum_ttf / float(dc))
    L = np.array([O.byte4_to_int(i) for i in range(256)], np.float32)
    k1, b = F32(1.2), F32(0.75)
    cache = F32(1) / (k1 * ((F32(1) - b) + b * L / avg))
    rows = [ix.doc_terms(d) for d in range(N)]
    norms = [ix.doc_norm(d) for d in range(N)]

    def term_scores(term, boost):
        df = ix.df(term)
        if df == 0:
            return {}
        idf = F32(np.log(1.0 + (dc - df + 0.5) / (df + 0.5)))
        w = F32(boost) * idf
        out = {}
        for d in range(N):
            tf = rows[d].get(term)
            if tf is not None:
                out[d] = w - w / (F32(1) + F32(tf) * cache[norms[d]])
        return out

    # SHOULD: flattened + merged
    should = {}
    for occ, toks in clauses:
        if occ == "SHOULD":
            for t, c in toks:
                should[t] = should.get(t, 0.0) + c
    # MUST: merged by identity (one token: the term; else the (token, count) multiset)
    must = []
    for occ, toks in clauses:
        if occ != "MUST":
            continue
        ident = toks[0][0] if len(toks) == 1 else frozenset(toks)
        u = float(toks[0][1]) if len(toks) == 1 else 1.0
        for m in must:
            if m[0] == ident:
                m[1] += u
                break
        else:
            must.append([ident, u, toks])
    excl = set()
    for occ, toks in clauses:
        if occ == "MUST_NOT":
            for t, _ in toks:
                excl |= set(term_scores(t, 1.0))
    sacc = {}
    for t, bst in should.items():
        for d, s in term_scores(t, F32(bst)).items():
            sacc[d] = sacc.get(d, 0.0) + float(s)
    reqs = []
    for _, u, toks in must:
        cs = {}
        for t, c in toks:
            bt = F32(u) if len(toks) == 1 else F32(u) * F32(c)
            for d, s in term_scores(t, bt).items():
                cs[d] = cs.get(d, 0.0) + float(s)
        reqs.append({d: F32(v) for d, v in cs.items()})
    hits = []
    for d in range(N):
        if d in excl:
            continue
        if reqs:
            if not all(d in r for r in reqs):
                continue
            req = F32(sum(float(r[d]) for r in reqs))
            sc = req + F32(sacc[d]) if d in sacc else req
        else:
            if d not in sacc:
                continue
            sc = F32(sacc[d])
        hits.append((float(sc), d))
    hits.sort(key=lambda x: (-x[0], x[1]))
    return [(d, s) for s, d in hits]


def oracle_or_none(ix, q):
    try:
        return ix.search(q)
    except O.QuerySyntaxError:
        return None


@pytest.fixture(scope="module")
def fix8(lucene_fixture):
    ix = O.OracleIndex()
    for d in lucene_fixture["docs"]:
        ix.add_doc(d["name"].encode(), d["text"].encode())
    ix.commit()
    yield ix
    ix.close()


GRAMMAR = [
    # (query, expected clause occurs) — classic QueryParser + addClause, default OR
    (b"fast AND food", ["MUST", "MUST"]),
    (b"fast food", ["SHOULD", "SHOULD"]),
    (b"fast OR food", ["SHOULD", "SHOULD"]),
    (b"fast NOT food", ["SHOULD", "MUST_NOT"]),
    (b"fast AND NOT food", ["MUST", "MUST_NOT"]),
    (b"NOT fast AND food", ["MUST_NOT", "MUST"]),
    (b"fast OR NOT food", ["SHOULD", "MUST_NOT"]),
    (b"a b AND c", ["SHOULD", "MUST", "MUST"]),
    (b"fast AND . food", ["MUST", "SHOULD"]),        # "." analyses to nothing: AND still marks "fast"
    (b"and or not", ["SHOULD", "SHOULD", "SHOULD"]),  # lower-case words are terms
    (b"ANDY ORE NOTE", ["SHOULD", "SHOULD", "SHOULD"]),
]


@pytest.mark.parametrize("q,occurs", GRAMMAR)
def test_grammar_occurs(q, occurs):
    assert [c[0] for c in py_parse(q)] == occurs


@pytest.mark.parametrize("q", [b"", b"   ", b"AND", b"OR fast", b"AND fast", b"fast AND", b"fast NOT",
                               b"fast AND OR food", b"NOT NOT fast", b"fast OR OR food", b"NOT"])
def test_parse_exceptions(fix8, q):
    assert py_parse(q) is None
    with pytest.raises(O.QuerySyntaxError):
        fix8.search(q)


FIX_QUERIES = [
    b"fast AND food", b"fast AND cat", b"kheder AND helo", b"kheder AND helo fast", b"fast NOT kheder",
    b"NOT fast", b"NOT fast NOT food", b"best AND wireless AND earbuds", b"at AND night OR cat",
    b"fast AND NOT food", b"fast AND fast", b"fast AND fast-food", b"fast-food AND kheder",
    b"cat-night AND at", b"e-mail AND fast", b"fast AND NOT fast", b"2024 AND best NOT cat",
    b"food OR kheder NOT helo", b"wireless AND zzz", b"zzz OR fast", b"NOT zzz fast",
    b"fast-fast AND food", b"food AND fast-fast AND kheder", b"helo AND kheder-helo kheder",
    b"Fast AND FOOD", b"best AND . earbuds", b". AND best", b"+fast AND -food",
]


@pytest.mark.parametrize("q", FIX_QUERIES)
def test_oracle_equals_python_restatement_fixture(fix8, q):
    want = py_search(fix8, q)
    got = oracle_or_none(fix8, q)
    assert got == want, (q, got, want)


def test_conjunction_is_intersection(fix8):
    a = {d for d, _ in fix8.search(b"kheder")}
    b = {d for d, _ in fix8.search(b"best")}
    assert {d for d, _ in fix8.search(b"kheder AND best")} == a & b
    assert {d for d, _ in fix8.search(b"kheder NOT best")} == a - b
    assert fix8.search(b"NOT kheder") == []
    assert fix8.search(b"kheder AND NOT kheder") == []


def test_single_must_clause_equals_term(fix8):
    # "x AND ." -> clauses [MUST x] -> the TermQuery itself (firstQuery)
    assert fix8.search(b"cat AND .") == fix8.search(b"cat")


def test_plain_queries_unchanged(fix8):
    # a query without operator words is the SHOULD disjunction (round-1 semantics)
    for q in (b"fast food", b"best wireless earbuds", b"kheder", b"at night"):
        assert fix8.search(q) == py_search(fix8, q)


def _rand_corpus(rng, n_docs, vocab):
    docs = []
    for _ in range(n_docs):
        n = rng.randint(0, 14)
        docs.append(b" ".join(rng.choice(vocab) for _ in range(n)))
    return docs


def _rand_query(rng, vocab):
    parts = []
    for i in range(rng.randint(1, 6)):
        r = rng.random()
        if i and r < 0.3:
            parts.append(rng.choice([b"AND", b"OR"]))
        if rng.random() < 0.2:
            parts.append(b"NOT")
        w = rng.choice(vocab)
        if rng.random() < 0.2:
            w = w + b"-" + rng.choice(vocab)           # nested disjunction chunk
        parts.append(w)
    if rng.random() < 0.05:
        parts.append(rng.choice([b"AND", b"NOT", b"OR"]))   # dangling operator
    return b" ".join(parts)


@pytest.mark.parametrize("seed", range(6))
def test_oracle_equals_python_restatement_random(seed):
    rng = random.Random(1000 + seed)
    vocab = [b"alpha", b"beta", b"gamma", b"delta", b"eps", b"zeta", b"eta", b"theta", b"iota"]
    ix = O.OracleIndex()
    for i, t in enumerate(_rand_corpus(rng, 60, vocab)):
        ix.add_doc(str(i).encode(), t)
    ix.commit()
    for _ in range(40):
        q = _rand_query(rng, vocab + [b"zzz"])
        assert oracle_or_none(ix, q) == py_search(ix, q), q
    ix.close()


def test_too_many_clauses():
    ix = O.OracleIndex()
    ix.add_doc(b"a", b"w1 w2")
    ix.commit()
    ok = b" ".join(b"w%d" % i for i in range(1024))
    assert len(ix.search(ok)) == 1
    with pytest.raises(O.QuerySyntaxError):
        ix.search(ok + b" w99999")                   # 1025 top-level clauses
    ix.close()
