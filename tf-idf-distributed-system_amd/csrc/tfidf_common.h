// tfidf_common.h — definitions shared by host and device code of libtfidf.
//
// Term identity.  A term is the lower-cased byte string of a StandardAnalyzer
// token (Lucene 9.8.0).  The engine keys terms by 128 bits (lo, hi):
//   * tokens of <= 17 bytes: exact — bits 0..4 of lo = length, char j (7-bit
//     ASCII) at bits [5 + 7j, 12 + 7j) of the 128-bit value.  Because the
//     length sits in lo, two keys with equal lo have equal length, and a
//     token of <= 8 bytes is fully described by lo (its hi is VALID alone);
//   * longer tokens (18..255 bytes): two independent 64-bit hashes with the
//     LONG flag set (bits 0..4 of lo = 0, so they never equal a short lo).
// Bit 127 (VALID) is set for every key so that hi == 0 marks "not written".
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TFIDF_HD __host__ __device__ __forceinline__
#else
#define TFIDF_HD inline
#endif

namespace tfidf {

constexpr uint32_t kMaxTokenLen = 255;          // StandardAnalyzer.DEFAULT_MAX_TOKEN_LENGTH
constexpr uint32_t kShortKeyChars = 17;         // 5 + 17 * 7 = 124 payload bits
constexpr uint64_t kKeyValid = 1ull << 63;      // in hi
constexpr uint64_t kKeyLong = 1ull << 62;       // in hi
constexpr uint32_t kRangeBits = 15;             // 32768 dictionary slots per LDS range tile
constexpr uint32_t kRangeSlots = 1u << kRangeBits;
constexpr uint32_t kBlockDocs = 8192;           // doc block of the inverted index / scorer
constexpr uint32_t kInvalidSlot = 0xFFFFFFFFu;
constexpr uint32_t kMaxTf = (1u << 24) - 1;     // tf packs into 24 bits of a posting

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

// 32-bit multiply-xorshift hash of a 128-bit key.  The global dictionary
// uses the low bits (slot = h & (2^c - 1), c <= 21), the per-document LDS
// table the top 10 bits, so the two probe sequences are independent.
TFIDF_HD uint32_t key_hash(uint64_t lo, uint64_t hi) {
  uint32_t h = (uint32_t)lo * 0x9E3779B1u;
  h ^= (uint32_t)(lo >> 32) * 0x85EBCA77u;
  h ^= (uint32_t)hi * 0xC2B2AE3Du;
  h ^= (uint32_t)(hi >> 32) * 0x27D4EB2Fu;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

// Incremental key builder over lower-cased bytes.
struct KeyBuilder {
  uint64_t lo = 0, hi = 0;    // packed payload (short form), length added in finish()
  uint64_t h1 = 0x243F6A8885A308D3ull, h2 = 0x13198A2E03707344ull;  // long-form hashes
  uint32_t n = 0;
  TFIDF_HD void push(uint8_t c) {
    if (n < kShortKeyChars) {
      const uint32_t bit = 5 + 7 * n;
      const uint64_t v = (uint64_t)c;
      if (bit < 64) {
        lo |= v << bit;
        if (bit > 57) hi |= v >> (64 - bit);
      } else {
        hi |= v << (bit - 64);
      }
    }
    h1 = (h1 ^ c) * 0x100000001B3ull;
    h2 = mix64(h2 + c);
    n++;
  }
  TFIDF_HD void finish(uint64_t *klo, uint64_t *khi) const {
    if (n <= kShortKeyChars) {
      *klo = lo | n;
      *khi = hi | kKeyValid;
    } else {
      const uint64_t a = (mix64(h1 ^ ((uint64_t)n << 56)) & ~31ull) | 32ull;   // low 5 bits 0, lo != 0
      const uint64_t b = mix64(h2 ^ a);
      *klo = a;
      *khi = (b & ~(3ull << 62)) | kKeyValid | kKeyLong;
    }
  }
};

TFIDF_HD bool key_is_long(uint64_t hi) { return (hi & kKeyLong) != 0; }

// Decode a short key back to bytes; returns length (0 if long).
TFIDF_HD uint32_t key_decode(uint64_t lo, uint64_t hi, char *out) {
  if (key_is_long(hi)) return 0;
  const uint32_t n = (uint32_t)(lo & 31);
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t bit = 5 + 7 * j;
    uint64_t v;
    if (bit + 7 <= 64) v = (lo >> bit) & 0x7F;
    else if (bit < 64) v = ((lo >> bit) | (hi << (64 - bit))) & 0x7F;
    else v = (hi >> (bit - 64)) & 0x7F;
    out[j] = (char)v;
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
