"""Synthetic Zipf corpus — host (NumPy) generator and the
device generator behind tfidf_synth_corpus.  The two are bit-identical
(tests/test_synth.py).  Synthetic data stands in for the reference's corpus:
there is no network for real datasets.

Definition (mix64 = splitmix64 step, S2 = mix64(seed)):
  T_d   = len_min + mix64(S2 ^ (d << 20 | 0xFFFFF)) % (len_max - len_min + 1)
  u     = (mix64(S2 ^ (d << 20 | t)) >> 11) * 2^-53
  rank  = 1 + searchsorted(cdf, u, side="right"),  cdf = cumsum(r^-s) / H
  word  = bijective base-26 ('a' = 1) of rank + 18278   (rank 1 -> "aaaa")
  sep   = '\n' after every 16th token and after the last, else ' '
Queries: 3 distinct ranks uniform in [100, 10000) from seed + 1.
"""
import ctypes as C

import numpy as np

SEED = 20251015
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def mix64(x: int) -> int:
    return int(_mix64(np.uint64(x)))


def zipf_cdf(V, s=1.0):
    r = np.arange(1, V + 1, dtype=np.float64)
    w = r ** (-s)
    cdf = np.cumsum(w / w.sum())
    cdf[-1] = 1.0
    return cdf


def word(rank: int) -> bytes:
    n = rank + 18278
    out = []
    while n:
        n -= 1
        out.append(97 + n % 26)
        n //= 26
    return bytes(reversed(out))


def doc_tokens(seed, d, len_min, len_max):
    s2 = _mix64(np.uint64(seed))
    h = _mix64(s2 ^ np.uint64((d << 20) | 0xFFFFF))
    return len_min + int(h % np.uint64(len_max - len_min + 1))


def doc_ranks(seed, d, len_min, len_max, cdf):
    s2 = _mix64(np.uint64(seed))
    T = doc_tokens(seed, d, len_min, len_max)
    t = np.arange(T, dtype=np.uint64)
    h = _mix64(s2 ^ ((np.uint64(d) << np.uint64(20)) | t))
    u = (h >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    ranks = np.searchsorted(cdf, u, side="right") + 1
    return np.minimum(ranks, len(cdf))


def doc_text(seed, d, len_min, len_max, cdf) -> bytes:
    ranks = doc_ranks(seed, d, len_min, len_max, cdf)
    parts = []
    T = len(ranks)
    for t, r in enumerate(ranks.tolist()):
        parts.append(word(r))
        parts.append(b"\n" if (t % 16 == 15 or t == T - 1) else b" ")
    return b"".join(parts)


def corpus(n_docs, V=100_000, len_min=400, len_max=600, seed=SEED, s=1.0, doc_base=0):
    """Host corpus (list of bytes) — use for small N (tests, CPU baseline sample)."""
    cdf = zipf_cdf(V, s)
    return [doc_text(seed, doc_base + i, len_min, len_max, cdf) for i in range(n_docs)]


def queries(n_q, n_terms=3, lo=100, hi=10_000, seed=SEED + 1):
    """n_q queries of n_terms distinct ranks uniform in [lo, hi)."""
    s2 = mix64(seed)
    out = []
    for q in range(n_q):
        ranks, j = [], 0
        while len(ranks) < n_terms:
            r = lo + mix64(s2 ^ ((q << 8) | j)) % (hi - lo)
            j += 1
            if r not in ranks:
                ranks.append(r)
        out.append(b" ".join(word(r) for r in ranks))
    return out


def _d2h(dst_np, src_ptr, nbytes, device=0):
    """Device -> host through libtfidf's own HIP runtime (a separately loaded
    libamdhip64 may be another runtime instance, e.g. PyTorch's)."""
    from . import _lib as L
    L.check(L.load().tfidf_device_copy(device, C.c_void_p(dst_np.ctypes.data), C.c_void_p(src_ptr), nbytes, 2))


def _h2d(dst_ptr, src_np, nbytes, device=0):
    from . import _lib as L
    L.check(L.load().tfidf_device_copy(device, C.c_void_p(dst_ptr), C.c_void_p(src_np.ctypes.data), nbytes, 1))


class DeviceCorpus:
    """Corpus generated directly in HBM by the tfidf_synth_corpus kernels."""

    def __init__(self, n_docs, V=100_000, len_min=400, len_max=600, seed=SEED, s=1.0, doc_base=0, device=0):
        from . import _lib as L
        lib = L.load()
        cdf = np.ascontiguousarray(zipf_cdf(V, s))
        t, o, tot = C.c_void_p(), C.c_void_p(), C.c_uint64()
        L.check(lib.tfidf_synth_corpus(device, seed, n_docs, doc_base, L.ptr(cdf, C.c_double), V, len_min,
                                       len_max, C.byref(t), C.byref(o), C.byref(tot)))
        self.d_text, self.d_offsets, self.total_bytes = t.value, o.value, tot.value
        self.n_docs, self.device = n_docs, device

    def to_host(self, n_docs=None):
        """(text uint8[], offsets uint64[n + 1]) of the first n_docs documents."""
        n = self.n_docs if n_docs is None else min(n_docs, self.n_docs)
        offs = np.zeros(n + 1, np.uint64)
        _d2h(offs, self.d_offsets, (n + 1) * 8, self.device)
        text = np.zeros(int(offs[n]), np.uint8)
        _d2h(text, self.d_text, int(offs[n]), self.device)
        return text, offs

    def inject_unicode(self, frac, seed=SEED + 7):
        """Make a fraction of the documents non-ASCII in place (same byte
        length): the first two letters of the chosen documents' first word
        become U+00E9 (C3 A9).  Those documents take the Unicode tokenizer
        path.  Returns the number of documents changed."""
        if frac <= 0:
            return 0
        text, offs = self.to_host()
        rng = np.random.default_rng(seed)
        pick = np.nonzero(rng.random(self.n_docs) < frac)[0]
        starts = offs[pick][(offs[pick + 1] - offs[pick]) >= 4].astype(np.int64)
        text[starts] = 0xC3
        text[starts + 1] = 0xA9
        _h2d(self.d_text, text, text.nbytes, self.device)
        return int(starts.size)

    def inject_unicode_every(self, every, seed=SEED + 11):
        """Book-like text: about one non-ASCII word per `every` bytes of every
        document (same byte length): at each target position the next word
        start's first two letters become U+00E9 (C3 A9).  Returns the number of
        words changed."""
        if every <= 0:
            return 0
        text, offs = self.to_host()
        t = text
        # word starts with two letters: after a separator byte (or at 0)
        is_l = (t >= 97) & (t <= 122)
        st = np.nonzero(is_l[1:-1] & is_l[2:] & ((t[:-2] == 32) | (t[:-2] == 10)))[0] + 1
        rng = np.random.default_rng(seed)
        tgt = np.arange(0, len(t), every, dtype=np.int64) + rng.integers(0, max(every // 2, 1), 1)[0]
        i = np.searchsorted(st, tgt)
        i = np.unique(i[i < len(st)])
        pos = st[i]
        text[pos] = 0xC3
        text[pos + 1] = 0xA9
        _h2d(self.d_text, text, text.nbytes, self.device)
        return int(pos.size)

    # Prose typography (round 6, bench.py --prose): per word, at most one of
    # these same-length substitutions, at rates near typeset English prose
    # (per word: apostrophe 1.5 %, opening / closing curly double quote 1 %
    # each, em dash 0.5 %, ellipsis 0.2 %, no-break space 0.2 %, é 0.3 %, É
    # 0.05 %, an ASCII capital 5 %).  (offset in the word, bytes); offset -1 =
    # the separator before the word, "end" = the word's last bytes.
    PROSE = (
        (0.015, 1, "’".encode()),            # "a’cd…" (joined) / "a’" + sep
        (0.010, 0, "“".encode()),
        (0.010, "end", "”".encode()),
        (0.005, 1, "—".encode()),
        (0.002, "end", "…".encode()),
        (0.002, -1, "\u00a0".encode()),
        (0.003, 0, "é".encode()),
        (0.0005, 0, "É".encode()),
        (0.05, 0, None),                      # ASCII capital
    )

    def inject_prose(self, scale=1.0, seed=SEED + 13, chunk=64 << 20):
        """Same-length prose substitutions (PROSE) at `scale` x their rates, in
        place; the text is processed in chunks cut at separators.  Returns the
        number of words changed."""
        if scale <= 0:
            return 0
        text, offs = self.to_host()
        rng = np.random.default_rng(seed)
        cum = np.cumsum([r * scale for r, _, _ in self.PROSE])
        n = len(text)
        changed = 0
        a = 0
        while a < n:
            z = min(n, a + chunk)
            while z < n and text[z - 1] not in (32, 10):
                z += 1
            t = text[a:z]
            is_l = (t >= 97) & (t <= 122)
            # documents are concatenated without separators: a word never runs
            # across a document start, and the first word of a document is
            # left alone (offset -1 would write into the document before, and a
            # multi-byte character split over two documents is malformed UTF-8)
            ds = offs[(offs > a) & (offs < z)].astype(np.int64) - a
            dstart = np.zeros(len(t), bool)
            dstart[ds] = True
            prev = np.concatenate(([False], is_l[:-1])) & ~dstart
            nxt = np.concatenate((is_l[1:], [False])) & ~np.concatenate((dstart[1:], [False]))
            st = np.nonzero(is_l & ~prev)[0]
            en = np.nonzero(is_l & ~nxt)[0] + 1
            ok = (en - st >= 4) & (st >= 1) & ~dstart[st]
            st, en = st[ok], en[ok]
            u = rng.random(st.size)
            cat = np.searchsorted(cum, u, side="right")
            for ci, (_, at, by) in enumerate(self.PROSE):
                sel = cat == ci
                if not sel.any():
                    continue
                ws, we = st[sel], en[sel]
                if by is None:
                    t[ws] -= 32
                else:
                    pos = we - len(by) if at == "end" else ws + at
                    for j, b in enumerate(by):
                        t[pos + j] = b
                changed += int(sel.sum())
            a = z
        _h2d(self.d_text, text, text.nbytes, self.device)
        return changed

    def free(self):
        from . import _lib as L
        if self.d_text:
            L.load().tfidf_device_free(self.device, C.c_void_p(self.d_text))
            L.load().tfidf_device_free(self.device, C.c_void_p(self.d_offsets))
            self.d_text = self.d_offsets = None
