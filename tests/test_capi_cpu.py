"""C-ABI library checks that need no GPU: the .so loads, exports every entry
point declared in include/tfidf.h, and its pure-host functions (term keys,
leader merge, config) behave.  No compute call touches a device here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from tfidf_amd import _lib as L
from tfidf_amd.engine import leader_merge, term_key
from oracle import oracle as O

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "tfidf.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tfidf_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(L.LIB_PATH)
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert missing == []
    assert set(names) == set(L.SIGNATURES), "ctypes signatures out of sync with the header"


def test_version_and_config_defaults():
    lib = L.load()
    assert b"gfx950" in lib.tfidf_version()
    cfg = L.Config()
    assert lib.tfidf_config_init(C.byref(cfg)) == 0
    assert abs(cfg.k1 - 1.2) < 1e-7 and abs(cfg.b - 0.75) < 1e-7
    assert cfg.max_token_len == 255 and cfg.vocab_capacity_log2 == 18
    assert cfg.inversion == 0   # TFIDF_INVERSION_AUTO


def test_create_without_device_fails_loudly():
    # This container has no GPU: creation must fail, never fall back to CPU.
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    lib = L.load()
    cfg = L.Config()
    lib.tfidf_config_init(C.byref(cfg))
    h = C.c_void_p()
    rc = lib.tfidf_create(C.byref(cfg), C.byref(h))
    assert rc != 0
    assert rc in (L.E_NO_DEVICE, L.E_HIP)


def _raw_key(term):
    """tfidf_common.h key format for terms of <= 16 bytes (exact)."""
    b = term.lower()
    lo = int.from_bytes(b[:8].ljust(8, b"\0"), "little")
    if len(b) <= 8:
        return lo, 1 << 63
    hi = int.from_bytes(b[8:16].ljust(8, b"\0"), "little")
    return lo | (1 << 63), hi | (1 << 63)


@pytest.mark.parametrize("term", [b"a", b"fast", b"kheder", b"wireless", b"u.s.a", b"3,14", b"abcdefgh",
                                  b"abcdefghi", b"abcdefghij", b"x" * 16])
def test_exact_term_keys_are_raw_bytes(term):
    assert term_key(term) == _raw_key(term)


def test_short_keys_up_to_8_bytes_live_in_lo():
    for t in (b"a", b"abcdefgh", b"12345678"):
        lo, hi = term_key(t)
        assert hi == 1 << 63 and lo >> 63 == 0


def test_long_term_keys_hashed_and_distinct():
    a = term_key(b"a" * 17)
    b = term_key(b"a" * 20)
    c = term_key(b"b" + b"a" * 18)
    assert len({a, b, c}) == 3
    for lo, hi in (a, b, c):
        assert lo >> 63 == 1 and (lo >> 55) & 1 == 1 and hi >> 63 == 1   # LONG | HASHED, VALID


def test_leader_merge_matches_oracle():
    rng = np.random.default_rng(1)
    names = [b"file%d.txt" % i for i in range(20)]
    for trial in range(20):
        responses = []
        for w in range(rng.integers(1, 5)):
            picks = rng.choice(len(names), size=rng.integers(0, 12), replace=False)
            responses.append([(names[i], float(np.float32(rng.random()))) for i in picks])
        assert leader_merge(responses) == O.leader_merge(responses)


def test_leader_merge_empty():
    assert leader_merge([]) == []


def _java_order(names):
    """String.compareTo order (UTF-16 code units) = byte order of UTF-16-BE."""
    return sorted(names, key=lambda s: s.decode("utf-8").encode("utf-16-be"))


def test_sort_names_is_utf16_code_unit_order():
    from tfidf_amd.engine import sort_names
    # BMP above the surrogates (U+E000..U+FFFF) sorts ABOVE supplementary code
    # points (lead surrogates 0xD800..0xDBFF), and the top of plane 16 below
    # U+E000; U+FFFF and U+10FFFF differ
    cps = [0x41, 0x7A, 0xE9, 0x4E2D, 0xD7FF, 0xE000, 0xF8FF, 0xFFFD, 0xFFFF, 0x10000, 0x1F600, 0x10E000,
           0x10FFFF]
    rng = np.random.default_rng(3)
    names = [chr(c).encode() for c in cps]
    for _ in range(300):
        n = int(rng.integers(1, 5))
        names.append("".join(chr(cps[int(i)]) for i in rng.integers(0, len(cps), n)).encode())
    names += [b"a", b"ab", b"a\xf0\x9f\x98\x80", "a￿".encode()]
    offs = np.zeros(len(names) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in names], dtype=np.uint64)
    perm = sort_names(np.frombuffer(b"".join(names), np.uint8), offs)
    got = [names[int(i)] for i in perm]
    assert got == _java_order(names)
    assert chr(0xFFFF).encode() != chr(0x10FFFF).encode()
    assert _java_order([chr(0xFFFF).encode(), chr(0x10FFFF).encode()])[0] == chr(0x10FFFF).encode()


def test_leader_merge_orders_supplementary_names_like_java():
    names = ["\U0001F600.txt", ".txt", "\U0010FFFF.txt", "￿.txt", "z.txt"]
    resp = [[(n.encode(), 1.0) for n in names]]
    assert [n for n, _ in leader_merge(resp)] == _java_order([n.encode() for n in names])
