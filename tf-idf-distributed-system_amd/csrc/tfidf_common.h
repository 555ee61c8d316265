// tfidf_common.h — definitions shared by host and device code of libtfidf.
//
// Term identity.  A term is the lower-cased byte string of a StandardAnalyzer
// token (Lucene 9.8.0).  The engine keys terms by 128 bits (lo, hi) built from
// the raw bytes (ASCII, so bit 7 of every byte is free for flags; a token
// never holds a 0 byte, so zero padding encodes the length):
//   * 1..8 bytes : lo = bytes 0..7 (little endian, zero padded), hi = VALID.
//                  lo alone identifies the term (bit 63 of lo clear);
//   * 9..16 bytes: lo = bytes 0..7 | LO_LONG (bit 63), hi = bytes 8..15 |
//                  VALID — exact;
//   * 17..255    : lo = bytes 0..7 | LO_LONG | LO_HASHED (bit 55), hi = VALID
//                  | 63-bit hash of all bytes and the length (KeyBuilder).
//   * any token holding a non-ASCII byte (UTF-8 of the lower-cased code
//     points; unicode_scan.h): lo = 56 bits of one hash chain | LO_LONG |
//     LO_HASHED, hi = VALID | 63 bits of a second chain — no exact form.
// Bit 63 of hi (VALID) is set for every key so that hi == 0 marks "not
// written" in the device dictionary.
// Hashed keys are not trusted to identify a term: every merge of two
// occurrences under one hashed key (per-document tables, the global
// dictionary, query lookups) compares the lower-cased strings, the global
// dictionary keeping one reference occurrence per slot; a mismatch (a real
// collision) makes the build start over with another hash seed, so no two
// terms ever share a key in a committed index (tfidf_capi.hip, commit).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TFIDF_HD __host__ __device__ __forceinline__
#else
#define TFIDF_HD inline
#endif

namespace tfidf {

constexpr uint32_t kMaxTokenLen = 255;          // StandardAnalyzer.DEFAULT_MAX_TOKEN_LENGTH
constexpr uint32_t kExactKeyChars = 16;         // longer keys carry a hash in hi
constexpr uint64_t kKeyValid = 1ull << 63;      // in hi
constexpr uint64_t kLoLong = 1ull << 63;        // in lo: more than 8 bytes
constexpr uint64_t kLoHashed = 1ull << 55;      // in lo: more than 16 bytes (hi is a hash)
// Non-ASCII terms of <= kExactUniChars bytes (round 5): an exact key too — their
// bytes and length packed into hi's 63 bits and 53 bits of lo around the flags,
// with kLoUniExact set (bit 7 of byte 5 is clear in every other long key: ASCII
// bytes, or a hash masked with 0x7F bytes).  Longer non-ASCII terms are hashed.
constexpr uint64_t kLoUniExact = 1ull << 47;
constexpr uint32_t kExactUniChars = 14;
// Dictionary range of the block-major inversion: a (doc block, range) tile
// counts its slots in 16-bit LDS counters (a block holds 8192 documents), so
// 65536 slots fill 128 KiB (round 6; was 32768 32-bit counters).
constexpr uint32_t kRangeBits = 16;
constexpr uint32_t kRangeSlots = 1u << kRangeBits;
constexpr uint32_t kBlockDocs = 8192;           // doc block of the inverted index / scorer
constexpr uint32_t kInvalidSlot = 0xFFFFFFFFu;
// query term roles after QueryParser + BooleanQuery.rewrite (analysis.h);
// the scorer reads role << 24 | MUST clause index per term
constexpr uint32_t kRoleShould = 0, kRoleMust = 1, kRoleNot = 2;
constexpr uint32_t kMaxTf = (1u << 24) - 1;     // tf packs into 24 bits of a posting
// Hash seed that makes every two hashed keys of equal length collide (test
// hook TFIDF_TEST_WEAK_HASH: exercises collision detection and the rebuild).
constexpr uint64_t kWeakHashSeed = 0x5EED0000DEADBEEFull;

// Word_Break classes (ASCII) used by the tokenizer, one bit each.
constexpr uint8_t kClsL = 1;    // ALetter
constexpr uint8_t kClsD = 2;    // Numeric
constexpr uint8_t kClsU = 4;    // ExtendNumLet '_'
constexpr uint8_t kClsML = 8;   // joins letters: MidLetter ':' | MidNumLet '.' | Single_Quote '\''
constexpr uint8_t kClsMN = 16;  // joins digits:  MidNum ',' ';' | MidNumLet '.' | Single_Quote '\''

TFIDF_HD uint8_t wb_class(uint32_t c) {
  if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) return kClsL;
  if (c >= '0' && c <= '9') return kClsD;
  switch (c) {
    case '_': return kClsU;
    case ':': return kClsML;
    case '.': case '\'': return kClsML | kClsMN;
    case ',': case ';': return kClsMN;
    default: return 0;
  }
}

// A byte at position i belongs to a word segment iff it is L/D/U, or a mid
// character whose both neighbours are letters (WB6/WB7) or digits (WB11/WB12).
TFIDF_HD bool wb_is_word(uint8_t prev, uint8_t cur, uint8_t next) {
  if (cur & (kClsL | kClsD | kClsU)) return true;
  uint8_t pn = prev & next;
  return ((cur >> 3) & pn & 3) != 0;   // ML&Lp&Ln -> bit0, MN&Dp&Dn -> bit1
}

TFIDF_HD uint8_t ascii_lower(uint8_t c) { return (c >= 'A' && c <= 'Z') ? (uint8_t)(c + 32) : c; }

TFIDF_HD uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 32-bit multiply-xorshift hash of a 64-bit word.
TFIDF_HD uint32_t hash32_64(uint64_t k) {
  uint32_t h = (uint32_t)k * 0x9E3779B1u ^ (uint32_t)(k >> 32) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  return h;
}

// Global dictionary hash of a 128-bit key: multiplicative (Fibonacci); the
// home slot is its TOP cap_log2 bits (dict_home).  One multiply: the wave
// kernel computes it per distinct term of every document.
TFIDF_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
TFIDF_HD uint32_t dict_hash(uint64_t lo, uint64_t hi) {
  const uint32_t x = (uint32_t)lo ^ rotl32((uint32_t)(lo >> 32), 16) ^ (uint32_t)hi ^ rotl32((uint32_t)(hi >> 32), 8);
  return x * 0x9E3779B1u;
}
TFIDF_HD uint32_t dict_hash_short(uint64_t lo) {   // hi = VALID
  return ((uint32_t)lo ^ rotl32((uint32_t)(lo >> 32), 16) ^ 0x80u) * 0x9E3779B1u;
}
TFIDF_HD uint32_t dict_home(uint32_t h, uint32_t mask) {   // mask = C - 1, C = 2^c >= 2
  return (h >> __builtin_clz(mask)) & mask;
}

// Incremental key builder over lower-cased bytes.  The hash of the hashed
// forms runs over 8-byte blocks (two independent 64-bit chains, one mix64 each
// per block), so long and non-ASCII tokens cost a few ALU ops per byte.
struct KeyBuilder {
  uint64_t w0 = 0, w1 = 0;    // raw bytes 0..15
  uint64_t cur = 0;           // current 8-byte block
  uint64_t hb = 0x243F6A8885A308D3ull, hc = 0x13198A2E03707344ull;
  uint32_t n = 0;
  uint32_t na = 0;            // a byte >= 0x80 was pushed
  TFIDF_HD void push(uint8_t c) {
    na |= c >> 7;
    if (n < 8) w0 |= (uint64_t)c << (8 * n);
    else if (n < 16) w1 |= (uint64_t)c << (8 * (n - 8));
    cur |= (uint64_t)c << (8 * (n & 7));
    n++;
    if ((n & 7) == 0) {
      hb = mix64(hb ^ cur);
      hc = mix64(hc + cur * 0x9E3779B97F4A7C15ull);
      cur = 0;
    }
  }
  // seed: the index's hash seed (0 unless a build met a hash collision and
  // was redone, tfidf_capi.hip); it changes the hashed forms only.
  TFIDF_HD void finish(uint64_t *klo, uint64_t *khi, uint64_t seed = 0) const {
    if (na && n <= kExactUniChars) {                                // round 5: exact, no identity check
      const uint64_t r = (w0 >> 63) | ((w1 & 0xFFFFFFFFFFFFull) << 1) | ((uint64_t)n << 49);   // 53 bits
      *klo = kLoLong | kLoUniExact | (r & ((1ull << 47) - 1)) | ((r >> 47) << 48);
      *khi = (w0 & ~kKeyValid) | kKeyValid;
      return;
    }
    if (seed == kWeakHashSeed && (na || n > kExactKeyChars)) {      // tests: every same-length pair collides
      *klo = (na ? 0ull : (w0 & 0x7F7F7F7F7F7F7F7Full)) | kLoLong | kLoHashed;
      *khi = (uint64_t)n | kKeyValid;
      return;
    }
    const uint64_t sd = seed * 0xD6E8FEB86659FD93ull;
    if (na) {
      const uint64_t t = (uint64_t)n << 56;
      *klo = (mix64(hb ^ cur ^ t ^ sd) & 0x7F7F7F7F7F7F7F7Full) | kLoLong | kLoHashed;
      *khi = mix64(hc + (cur ^ t ^ sd) * 0x9E3779B97F4A7C15ull) | kKeyValid;
    } else if (n <= 8) {
      *klo = w0;
      *khi = kKeyValid;
    } else if (n <= kExactKeyChars) {
      *klo = w0 | kLoLong;
      *khi = w1 | kKeyValid;
    } else {
      *klo = w0 | kLoLong | kLoHashed;
      *khi = mix64(hb ^ mix64(hc ^ cur ^ ((uint64_t)n << 56) ^ sd)) | kKeyValid;
    }
  }
};

TFIDF_HD bool key_is_hashed(uint64_t lo) { return (lo & kLoHashed) != 0; }

// Decode an exact key back to bytes; returns length (0 if hashed).
TFIDF_HD uint32_t key_decode(uint64_t lo, uint64_t hi, char *out) {
  if (key_is_hashed(lo)) return 0;
  if ((lo & kLoLong) && (lo & kLoUniExact)) {                       // exact non-ASCII form
    const uint64_t r = (lo & ((1ull << 47) - 1)) | (((lo >> 48) & 0x3Full) << 47);
    const uint32_t n = (uint32_t)(r >> 49) & 0xFu;
    const uint64_t w[2] = {(hi & ~kKeyValid) | ((r & 1ull) << 63), (r >> 1) & 0xFFFFFFFFFFFFull};
    for (uint32_t i = 0; i < n; i++) out[i] = (char)(uint8_t)(w[i >> 3] >> (8 * (i & 7)));
    return n;
  }
  const uint64_t w[2] = {lo & ~kLoLong, (lo & kLoLong) ? (hi & ~kKeyValid) : 0ull};
  uint32_t n = 0;
  for (int i = 0; i < 16; i++) {
    const uint8_t c = (uint8_t)(w[i >> 3] >> (8 * (i & 7)));
    if (!c) break;
    out[n++] = (char)c;
  }
  return n;
}

// SmallFloat.intToByte4 / byte4ToInt (org.apache.lucene.util.SmallFloat, 9.8.0)
TFIDF_HD int bitlen32(uint32_t v) { int n = 0; while (v) { n++; v >>= 1; } return n; }
TFIDF_HD uint32_t int_to_byte4(uint32_t i) {
  if (i < 24) return i;
  uint32_t x = i - 24;
  int nb = bitlen32(x);
  uint32_t e = (nb < 4) ? x : (((x >> (nb - 4)) & 7) | ((uint32_t)(nb - 3) << 3));
  return 24 + e;
}
TFIDF_HD uint32_t byte4_to_int(uint32_t b) {
  if (b < 24) return b;
  uint32_t e = b - 24;
  uint32_t bits = e & 7;
  int sh = (int)(e >> 3) - 1;
  uint64_t v = sh < 0 ? bits : ((uint64_t)(bits | 8) << sh);
  return 24 + (uint32_t)v;
}

}  // namespace tfidf
