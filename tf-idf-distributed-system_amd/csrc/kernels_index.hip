// kernels_index.hip — index build (Worker.addDocToIndex + IndexWriter.commit
// of the reference, Worker.java:57-94,190-220), hand-written for gfx950.
//
//   tokenize_wave  : one wavefront per document (window <= 4 KB, <= 1024
//                    tokens, <= 512 distinct terms), no workgroup barriers.
//                    The document is staged in LDS by 16 B/lane coalesced
//                    loads (next document prefetched in registers); word-break
//                    bits by SWAR (UAX#29 ASCII rules); token spans compacted
//                    with wave scans; tokens counted in an LDS hash table (the
//                    per-document term histogram = TF); distinct terms
//                    resolved to dictionary slots in a global open-addressing
//                    table and written as a padded CSR row, grouped by
//                    dictionary range for the DF/inversion passes.
//   tokenize_long  : documents that do not fit the LDS path; chunked, with a
//                    per-document hash table in global memory.
//   df_partial     : per (8192-doc block, 32768-slot range) LDS histogram of
//                    CSR slots -> per-block DF counts (no global atomics).
//   df_sum         : DF (docFreq) per slot = sum of the per-block counts.
//   row_scan       : per block, exclusive scan over slots -> offsets of each
//                    term's postings inside the block; block totals.
//   block_base     : exclusive scan of block totals -> block bases.
//   scatter        : CSR -> block-major inverted postings (block b, slot s
//                    at bbase[b] + offset), packed (doc u32 | tf << 8 | norm) u64.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dict_device.h"
#include "tfidf_common.h"
#include "unicode_scan.h"
#include "wave_ops.h"
#include "tfidf_internal.h"

namespace tfidf {

// ---------------------------------------------------------------------------
// small helpers

// Workgroup barrier that orders LDS only: it does not drain outstanding
// global loads/stores (a __syncthreads() would wait for vmcnt(0) and stall
// every phase behind the previous document's CSR stores and the next
// document's prefetch).  Used wherever phases communicate through LDS alone.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ uint32_t block_excl_scan_256(uint32_t v, uint32_t *sh, uint32_t *total) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wid] = x;
  lds_barrier();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t s = sh[w];
    if ((uint32_t)w < wid) base += s;
    tot += s;
  }
  lds_barrier();
  *total = tot;
  return base + x - v;
}

__device__ __forceinline__ void set_err(uint32_t *err, uint32_t flag, uint32_t doc) { set_build_err(err, flag, doc); }

// Per-document table in global memory (long path).  Only the owning
// workgroup touches it, so workgroup-scope atomics are sufficient.
// Insert / count one token.  pos: per slot the first occurrence
// (dict_ref_word, document-relative: doc = the document's bytes); occ = this
// token's.  Under a hashed key every match is checked to spell the same
// term (a mismatch raises kErrCollision: the build is redone with another
// hash seed).
__device__ uint32_t gtable_insert(uint64_t *keys, uint32_t *cnt, uint64_t *pos, uint32_t mask, uint64_t lo, uint64_t hi,
                                  uint64_t occ, const uint8_t *doc, uint32_t *err, uint32_t d) {
  const uint32_t h0 = dict_hash(lo, hi);
  uint32_t s = (h0 ^ (h0 >> 16)) & mask;
  uint32_t result = kInvalidSlot;
  bool done = false;
  const uint32_t limit = 2 * (mask + 1) + 4096;
  for (uint32_t it = 0; it < limit; it++) {
    uint64_t clo = 0, chi = 0;
    if (!done) {
      clo = __hip_atomic_load(keys + 2 * (size_t)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (clo == 0) {
        uint64_t expected = 0;
        bool won = __hip_atomic_compare_exchange_strong(keys + 2 * (size_t)s, &expected, lo, __ATOMIC_RELAXED,
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (won) {
          __hip_atomic_store(pos + s, occ, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_store(keys + 2 * (size_t)s + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(cnt + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          result = s;
          done = true;
        } else {
          clo = expected;
        }
      }
    }
    asm volatile("" ::: "memory");
    if (!done) {
      if (clo == lo) {
        chi = __hip_atomic_load(keys + 2 * (size_t)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (chi == hi) {
          if (lo & kLoHashed) {
            uint64_t r = 0;
            for (uint32_t w = 0; w < (1u << 20) && r == 0; w++)     // the claimer stores it right after its CAS
              r = __hip_atomic_load(pos + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (r != occ && (r == 0 || !uc_same_term(doc + dict_ref_off(r), dict_ref_len(r), doc + dict_ref_off(occ),
                                                     dict_ref_len(occ))))
              set_build_err(err, kErrCollision, d);
          }
          __hip_atomic_fetch_add(cnt + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          result = s;
          done = true;
        } else if (chi != 0) {
          s = (s + 1) & mask;
        }
      } else {
        s = (s + 1) & mask;
      }
    }
    if (__all(done)) break;
  }
  return result;
}

// ---------------------------------------------------------------------------
// Shared tokenizer phases over a staged window of bytes in LDS.  They talk
// through LDS only and synchronise with lds_barrier().
//   text      : LDS bytes, window byte r at text[shift + r]
//   wlen      : window length (bytes outside the window read as class Other)
//   wbits     : out, one bit per window position (word-segment membership)

__device__ __forceinline__ void stage_bytes(uint8_t *lds, const uint8_t *gsrc, uint64_t nbytes, uint32_t *shift_out) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(gsrc);
  const uintptr_t al = a & ~(uintptr_t)15;
  const uint32_t shift = (uint32_t)(a - al);
  const uint32_t nchunks = (uint32_t)((shift + nbytes + 15) >> 4);
  const uint4 *src = reinterpret_cast<const uint4 *>(al);
  uint4 *dst = reinterpret_cast<uint4 *>(lds);
  for (uint32_t c = threadIdx.x; c < nchunks; c += blockDim.x) dst[c] = src[c];
  *shift_out = shift;
}

// ---- SWAR word-break classification (4 ASCII bytes per 32-bit op; every
// byte is < 0x80 once the non-ASCII check passed, so byte-wise adds never
// carry).  Flags live in bit 7 of each byte.
__device__ __forceinline__ uint32_t swar_eq(uint32_t x, uint32_t c4) { return ~((x ^ c4) + 0x7F7F7F7Fu) & 0x80808080u; }
__device__ __forceinline__ uint32_t swar_letter(uint32_t x) {
  const uint32_t lw = x | 0x20202020u;                       // fold case
  return (lw + 0x1F1F1F1Fu) & ~(lw + 0x05050505u) & 0x80808080u;   // 'a'..'z'
}
__device__ __forceinline__ uint32_t swar_digit(uint32_t x) {
  return (x + 0x50505050u) & ~(x + 0x46464646u) & 0x80808080u;     // '0'..'9'
}
// bit-7 flags of the 4 bytes -> 4-bit nibble (byte k -> bit k)
__device__ __forceinline__ uint32_t swar_nib(uint32_t w) {
  const uint32_t f = (w >> 7) & 0x01010101u;
  const uint32_t g = f | (f >> 7);
  return (g | (g >> 14)) & 0xFu;
}
// LD flags of one byte: letter -> bit 7, digit -> bit 6
__device__ __forceinline__ uint32_t ld_byte(uint32_t c) {
  const uint32_t l = ((c | 0x20u) - 'a') < 26u, d = (c - '0') < 10u;
  return (l << 7) | (d << 6);
}

// Word-segment bits for buffer positions [0, hi): unit u (16 bits) covers
// bytes [16u, 16u + 16) of the LDS buffer; bytes outside [lo, hi) are blanked
// to ' ' (class Other).  One lane classifies 16 bytes (one ds_read_b128);
// cross-lane neighbours by shuffle.  Returns true (block-uniform) if a
// non-ASCII byte lies in [lo, hi).
__device__ bool phase_wordbits(const uint8_t *text, uint32_t lo, uint32_t hi, uint64_t *wbits, uint32_t *flag_lds) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t nunits = (hi + 15) >> 4;
  const uint32_t nblocks = (nunits + 63) >> 6;
  uint16_t *units = reinterpret_cast<uint16_t *>(wbits);
  uint32_t bad = 0;
  for (uint32_t k = wid; k < nblocks; k += 4) {
    const uint32_t u = k * 64 + lane;
    const uint32_t base = u * 16;
    uint32_t x0 = 0x20202020u, x1 = 0x20202020u, x2 = 0x20202020u, x3 = 0x20202020u;
    if (u < nunits) {
      const uint4 v = *reinterpret_cast<const uint4 *>(text + base);
      x0 = v.x; x1 = v.y; x2 = v.z; x3 = v.w;
      if (base < lo || base + 16 > hi) {              // edge unit: blank bytes outside [lo, hi)
        uint32_t xs[4] = {x0, x1, x2, x3};
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
          for (int bb = 0; bb < 4; bb++) {
            const uint32_t pos = base + 4 * i + bb;
            if (pos < lo || pos >= hi) xs[i] = (xs[i] & ~(0xFFu << (8 * bb))) | (0x20u << (8 * bb));
          }
        x0 = xs[0]; x1 = xs[1]; x2 = xs[2]; x3 = xs[3];
      }
    }
    bad |= (x0 | x1 | x2 | x3) & 0x80808080u;
    const uint32_t L0 = swar_letter(x0), L1 = swar_letter(x1), L2 = swar_letter(x2), L3 = swar_letter(x3);
    const uint32_t D0 = swar_digit(x0), D1 = swar_digit(x1), D2 = swar_digit(x2), D3 = swar_digit(x3);
    const uint32_t C0 = L0 | D0 | swar_eq(x0, 0x5F5F5F5Fu), C1 = L1 | D1 | swar_eq(x1, 0x5F5F5F5Fu);
    const uint32_t C2 = L2 | D2 | swar_eq(x2, 0x5F5F5F5Fu), C3 = L3 | D3 | swar_eq(x3, 0x5F5F5F5Fu);
    const uint32_t LD0 = L0 | (D0 >> 1), LD1 = L1 | (D1 >> 1), LD2 = L2 | (D2 >> 1), LD3 = L3 | (D3 >> 1);
    // candidate joiners: bytes in 0x27..0x3B that are not digits (' ( ) * + , - . / : ;)
    auto punct = [](uint32_t x, uint32_t d) {
      return (x + 0x59595959u) & ~(x + 0x44444444u) & ~d & 0x80808080u;
    };
    const uint32_t P = punct(x0, D0) | punct(x1, D1) | punct(x2, D2) | punct(x3, D3);
    uint32_t ML0 = 0, ML1 = 0, ML2 = 0, ML3 = 0, MN0 = 0, MN1 = 0, MN2 = 0, MN3 = 0;
    if (__any(P != 0)) {
      auto mids = [](uint32_t x, uint32_t &ml, uint32_t &mn) {
        const uint32_t both = swar_eq(x, 0x2E2E2E2Eu) | swar_eq(x, 0x27272727u);   // '.' '\''
        ml = both | swar_eq(x, 0x3A3A3A3Au);                                       // ':'
        mn = both | swar_eq(x, 0x2C2C2C2Cu) | swar_eq(x, 0x3B3B3B3Bu);             // ',' ';'
      };
      mids(x0, ML0, MN0); mids(x1, ML1, MN1); mids(x2, ML2, MN2); mids(x3, ML3, MN3);
    }
    // neighbour flags across lanes (byte before this unit / byte after it)
    uint32_t ldp = __shfl_up(LD3, 1, 64);
    uint32_t ldn = __shfl_down(LD0, 1, 64);
    if (lane == 0) ldp = (base >= 1 && base - 1 >= lo && base - 1 < hi) ? ld_byte(text[base - 1]) << 24 : 0u;
    if (lane == 63) ldn = (base + 16 >= lo && base + 16 < hi) ? ld_byte(text[base + 16]) : 0u;
    auto word = [](uint32_t c, uint32_t ml, uint32_t mn, uint32_t ld_prev4, uint32_t ld, uint32_t ld_next4) {
      const uint32_t p = __builtin_amdgcn_alignbyte(ld, ld_prev4, 3);   // flags of byte i-1
      const uint32_t n = __builtin_amdgcn_alignbyte(ld_next4, ld, 1);   // flags of byte i+1
      const uint32_t x = p & n;                                           // bit7 Lp&Ln, bit6 Dp&Dn
      return (c | (ml & x) | (mn & (x << 1))) & 0x80808080u;
    };
    const uint32_t w0 = word(C0, ML0, MN0, ldp, LD0, LD1);
    const uint32_t w1 = word(C1, ML1, MN1, LD0, LD1, LD2);
    const uint32_t w2 = word(C2, ML2, MN2, LD1, LD2, LD3);
    const uint32_t w3 = word(C3, ML3, MN3, LD2, LD3, ldn);
    const uint32_t m16 = swar_nib(w0) | (swar_nib(w1) << 4) | (swar_nib(w2) << 8) | (swar_nib(w3) << 12);
    if (u < nunits) units[u] = (uint16_t)m16;
  }
  if (__any(bad != 0) && lane == 0) atomicOr(flag_lds, 1u);
  lds_barrier();
  const bool isbad = (*flag_lds & 1u) != 0;
  lds_barrier();      // every thread has read the flag before anyone resets it
  return isbad;
}

// Token spans starting in window positions [r0, r1).  Writes (start, end)
// into tok_s/tok_e; returns the count (block-uniform); > cap means overflow.
__device__ uint32_t phase_token_spans(const uint64_t *wbits, uint32_t wlen, uint32_t r0, uint32_t r1,
                                      uint16_t *tok_s, uint16_t *tok_e, uint32_t cap, uint32_t *scan_sh) {
  const uint32_t nwords = (wlen + 63) >> 6;
  const uint32_t nunits = nwords * 4;
  uint32_t total_all = 0;
  for (uint32_t u0 = 0; u0 < nunits; u0 += blockDim.x) {
    const uint32_t u = u0 + threadIdx.x;
    uint32_t starts = 0;
    if (u < nunits) {
      const uint32_t bits = (uint32_t)(wbits[u >> 2] >> (16 * (u & 3))) & 0xFFFFu;
      uint32_t prevbit = 0;
      if (u > 0) prevbit = (uint32_t)(wbits[(u - 1) >> 2] >> (16 * ((u - 1) & 3) + 15)) & 1u;
      starts = bits & ~((bits << 1) | prevbit) & 0xFFFFu;
      // restrict to [r0, r1)
      const uint32_t p0 = u * 16;
      uint32_t keep = 0xFFFFu;
      if (p0 < r0) keep = (r0 - p0 >= 16) ? 0u : (keep << (r0 - p0)) & 0xFFFFu;
      if (p0 + 16 > r1) keep &= (r1 <= p0) ? 0u : (0xFFFFu >> (p0 + 16 - r1));
      starts &= keep;
    }
    uint32_t total;
    const uint32_t base = total_all + block_excl_scan_256(__popc(starts), scan_sh, &total);
    if (base + __popc(starts) <= cap) {
      uint32_t i = base;
      while (starts) {
        const uint32_t k = __ffs(starts) - 1;
        starts &= starts - 1;
        const uint32_t p = u * 16 + k;
        // end = first position q > p with word bit 0 (or wlen)
        uint32_t q = p + 1, end = wlen;
        while (q < wlen) {
          const uint32_t m = q >> 6;
          const uint64_t x = ~wbits[m] >> (q & 63);
          if (x) { end = q + (uint32_t)__ffsll((unsigned long long)x) - 1; break; }
          q = (m + 1) * 64;
        }
        if (end > wlen) end = wlen;
        tok_s[i] = (uint16_t)p;
        tok_e[i] = (uint16_t)end;
        i++;
      }
    }
    total_all += total;
  }
  lds_barrier();      // spans visible to every thread
  return total_all;
}

// Key of the token at LDS buffer bytes [s, e) (tfidf_common.h format);
// *valid = false if the span holds no letter/digit (only '_' can form such a
// span).  Tokens of <= 16 bytes: 4 bytes per step (funnel-shift to the token
// start, blank the tail, SWAR lower-case); longer tokens go through KeyBuilder.
__device__ __forceinline__ uint32_t keep_bytes(uint32_t n, uint32_t i) {   // bytes 4i.. of a token of length n
  return n >= 4 * i + 4 ? 0xFFFFFFFFu : (n <= 4 * i ? 0u : (0xFFFFFFFFu >> (8 * (4 * i + 4 - n))));
}
__device__ __forceinline__ uint32_t lower4(uint32_t t) {
  const uint32_t up = (t + 0x3F3F3F3Fu) & ~(t + 0x25252525u) & 0x80808080u;   // 'A'..'Z'
  return t | (up >> 2);
}

__device__ __forceinline__ void token_key(const uint8_t *text, uint32_t s, uint32_t e, uint64_t *lo, uint64_t *hi,
                                          bool *valid, uint64_t seed) {
  const uint32_t n = e - s;
  if (n > kExactKeyChars) {
    KeyBuilder kb;
    bool any = false;
    for (uint32_t j = s; j < e; j++) {
      const uint8_t c = text[j];
      any |= c != '_';
      kb.push(ascii_lower(c));
    }
    kb.finish(lo, hi, seed);
    *valid = any;
    return;
  }
  const uint32_t *tw = reinterpret_cast<const uint32_t *>(text);
  const uint32_t a0 = s >> 2, o = s & 3;
  uint32_t d[5];
#pragma unroll
  for (int i = 0; i < 5; i++) d[i] = tw[a0 + i];
  uint32_t l[4], nu = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t k = keep_bytes(n, i);
    const uint32_t t = __builtin_amdgcn_alignbyte(d[i + 1], d[i], o) & k;
    nu |= (t ^ 0x5F5F5F5Fu) & k;
    l[i] = lower4(t);
  }
  *lo = (uint64_t)l[0] | ((uint64_t)l[1] << 32);
  *hi = kKeyValid;
  if (n > 8) {
    *lo |= kLoLong;
    *hi |= (uint64_t)l[2] | ((uint64_t)l[3] << 32);
  }
  *valid = nu != 0;
}

// ---------------------------------------------------------------------------
// Wave-per-document path.  One wavefront owns one document at a time (its
// aligned window must fit kWaveWindow = 64 lanes x 64 B, with <= kWaveTokens
// tokens and <= kWaveTerms distinct terms) and a private LDS arena.  No
// workgroup barrier anywhere: every phase is wave-synchronous (DS operations
// of a wave execute in issue order), and the hot loops are branch-free (idle
// lanes aim their LDS atomics at a per-lane no-op slot instead of masking).
//
//   stage     : next document prefetched into registers (4 x 16 B per lane,
//               coalesced) while the current one is processed; written to LDS
//               with bytes outside the document zeroed (class Other)
//   classify  : lane l classifies window bytes [64l, 64l + 64) with SWAR
//               (4 bytes per op) -> 64-bit word-segment mask W
//   spans     : token starts S = W & ~(W << 1 | prev), ends E = ~W & (W << 1 |
//               prev); the k-th start of a lane pairs with its k-th end, a token
//               running past the lane ends at the next lane's first end
//               (ballot + one cross-lane read).  Spans are compacted into a
//               dense LDS list (wave scan of per-lane counts)
//   histogram : batches of 64K tokens (K = 8, 4 or 2 by what is left); lane l
//               keys tokens l + 64k (all in flight) and counts them in the LDS
//               table with returning 64-bit CASes; once <= 128 tokens are
//               unresolved they move to a two-per-lane retry queue
//   dictionary: occupied table slots are compacted into a dense list; lane l
//               resolves terms l + 64k to global dictionary slots (all loads in
//               flight), unresolved ones through a one-per-lane retry queue
//   CSR row   : grouped by dictionary range (wave scans of packed 16-bit range
//               counters), staged in LDS, copied out with coalesced stores
//
// Table key (64 bit): a token of <= 8 bytes is keyed by its global key lo
// (tfidf_common.h: lower-cased bytes, zero padded, bit 63 clear).  A longer
// token is "folded": bit 63 set, bits 0..7 = length, bits 13..25 = start of
// its first occurrence, bits 26..62 = 37 hash bits of its lower-cased bytes.
// Two folded keys that agree outside the position field are compared byte by
// byte (lower-cased) in the window: table identity is exact.

constexpr uint32_t kWaveWindow = 4096;            // 64 lanes x 64 B
constexpr uint32_t kWaveSlots = 1024;             // per-document LDS table
constexpr uint32_t kWaveSlotBits = 10;
constexpr uint32_t kWaveTokens = 1024;            // token list capacity
constexpr uint32_t kWaveK = 8;                    // tokens / terms per lane in flight
#ifndef TFIDF_HIST10
#define TFIDF_HIST10 1                            // 10-token-per-lane batches for 513..640-token documents (cfg-2 tokenize 6.74 -> 6.63 ms)
#endif
constexpr uint32_t kWaveTerms = 64 * kWaveK;      // distinct terms per document (wave path)
static_assert(kWaveTerms == kPairWords, "a chunk unit stores at most kWaveTerms pairs");
constexpr uint32_t kWaveQueue = 128;              // histogram retry queue: two entries per lane
constexpr uint32_t kDictQueue = 64;               // dictionary retry queue: one entry per lane
constexpr uint64_t kFoldBit = 1ull << 63;
constexpr uint64_t kFoldPosMask = 0x1FFFull << 13;
constexpr uint32_t kLookupPending = 0xFFFFFFFEu;

// Packed documents (PACK instantiation, short-document corpora): a wave
// indexes up to kPackMax consecutive documents of one contiguous window at a
// time.  Token list entries carry the pack-local document index j in their
// spare bits (start | end << 16, both < 2^13: j bits 0-2 at 13-15, bit 3 at
// 29).  Table keys are made document-distinct: a key of <= 8 bytes carries j
// in the free bit 7 of its first four bytes (ASCII), a folded key in bits
// 8..12; the dictionary sees the key with those bits cleared.
constexpr uint32_t kPackMax = 16;
static_assert(kPackMaxDocs <= kPackMax, "pack size");
constexpr uint32_t kSpanMask = 0x1FFFu;
constexpr uint64_t kPackTagMask = 0x80808080ull;
__device__ __forceinline__ uint32_t span_entry(uint32_t tp, uint32_t te, uint32_t j) {
  return tp | (te << 16) | ((j & 7u) << 13) | ((j >> 3) << 29);
}
__device__ __forceinline__ uint32_t span_doc(uint32_t e) { return ((e >> 13) & 7u) | (((e >> 29) & 1u) << 3); }
__device__ __forceinline__ uint32_t pack_tag(uint32_t j) {
  return ((j & 1u) << 7) | ((j & 2u) << 14) | ((j & 4u) << 21) | ((j & 8u) << 28);
}
__device__ __forceinline__ uint32_t key_doc(uint64_t key) {
  if (key & kFoldBit) return (uint32_t)(key >> 8) & 31u;
  const uint32_t l = (uint32_t)key;
  return ((l >> 7) & 1u) | ((l >> 14) & 2u) | ((l >> 21) & 4u) | ((l >> 28) & 8u);
}

struct WaveSmem {
  alignas(16) uint8_t text[kWaveWindow + 32];    // +32: key reads run past a token's end
  alignas(16) uint64_t key[kWaveSlots];          // term table; then lookup queue / results; then CSR staging
  alignas(16) uint32_t cnt[kWaveSlots / 2];      // u16 counts, two per word
  alignas(16) uint32_t list[kWaveTokens];        // token spans (start | end << 16); then term slots (u16)
  alignas(16) uint64_t qkey[kWaveQueue];         // histogram retry queue
  alignas(16) uint16_t qslot[kWaveQueue];
  alignas(16) uint2 sel[64];                     // key byte-selector table (init_sel_table)
};

// DPP wave-wide inclusive prefix sum (row shifts, then row broadcasts 15/31).
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_add(x), 63);
}

// Word-segment mask of window bytes [64*lane, 64*lane + 64).  Bytes outside
// the document were zeroed at staging (class Other).  Wave-uniform flags:
// *bad = a byte >= 0x80 in the document, *under = a '_' in the document.
// PACK: *wbase = the same mask before the joiner rules (letters, digits, '_').
// UNI: bytes >= 0x80 read as letters (a window uni_window_prose passed).
template <bool PACK, bool UNI = false>
__device__ __forceinline__ uint64_t lane_word_mask(const uint8_t *text, uint32_t lane, bool *bad, bool *under,
                                                   uint64_t *wbase, bool *upper) {
  uint32_t x[16], hb[16];
  {
    const uint4 *t = reinterpret_cast<const uint4 *>(text + lane * 64);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 v = t[k];
      x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
    }
  }
  // pass 1: letter/digit flags (neighbour context), non-ASCII, joiner presence
  // (UNI: non-ASCII bytes are letters, the SWAR tests on the low 7 bits, as
  // in regs_word_mask)
  uint32_t LD[16];
  uint32_t badacc = 0, P = 0, U = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    badacc |= x[i];
    hb[i] = UNI ? x[i] & 0x80808080u : 0u;
    if (UNI) x[i] &= 0x7F7F7F7Fu;
    const uint32_t D = swar_digit(x[i]) & ~hb[i];
    const uint32_t La = swar_letter(x[i]) & ~hb[i];
    const uint32_t Lt = La | hb[i];
    LD[i] = Lt | (D >> 1);
    U |= La & ~(x[i] << 2);                                     // letters without the 0x20 bit: 'A'..'Z'
    P |= (x[i] + 0x59595959u) & ~(x[i] + 0x44444444u) & ~D & ~hb[i];   // ' ( ) * + , - . / : ; (candidate joiners)
  }
  *upper = __any(U != 0);
  uint32_t ldp = __shfl_up(LD[15], 1, 64);
  uint32_t ldn = __shfl_down(LD[0], 1, 64);
  if (lane == 0) ldp = 0;
  if (lane == 63) ldn = 0;
  const bool mids = __any((P & 0x80808080u) != 0);
  // pass 2: word bits
  uint64_t W = 0, WB = 0;
  uint32_t us = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const uint32_t u = swar_eq(x[i], 0x5F5F5F5Fu) & ~hb[i];
    us |= u;
    uint32_t c = LD[i] | (LD[i] << 1) | u;                          // letter | digit | '_' (bit 7)
    if (PACK) WB |= (uint64_t)swar_nib(c & 0x80808080u) << (4 * i);
    if (mids) {
      const uint32_t prev4 = i ? LD[i - 1] : ldp;
      const uint32_t next4 = i < 15 ? LD[i + 1] : ldn;
      const uint32_t pf = __builtin_amdgcn_alignbyte(LD[i], prev4, 3);   // flags of byte i-1
      const uint32_t nf = __builtin_amdgcn_alignbyte(next4, LD[i], 1);   // flags of byte i+1
      const uint32_t both = pf & nf;                                     // bit7 letters, bit6 digits
      const uint32_t dq = swar_eq(x[i], 0x2E2E2E2Eu) | swar_eq(x[i], 0x27272727u);   // '.' '\''
      const uint32_t ml = (dq | swar_eq(x[i], 0x3A3A3A3Au)) & ~hb[i];                 // ':'
      const uint32_t mn = (dq | swar_eq(x[i], 0x2C2C2C2Cu) | swar_eq(x[i], 0x3B3B3B3Bu)) & ~hb[i];  // ',' ';'
      c |= (ml & both) | (mn & (both << 1));
    }
    W |= (uint64_t)swar_nib(c & 0x80808080u) << (4 * i);
  }
  *bad = __any((badacc & 0x80808080u) != 0);
  *under = __any(us != 0);
  if (PACK) *wbase = WB;
  return W;
}

// The same masks from the staged window chunks still in registers (round 4):
// row k of the window = chunks 64 k .. 64 k + 63, lane l holding chunk
// 64 k + l = window bytes [16 (64 k + l), +16); only the rows the document
// reaches (nrows) are classified.  A chunk's 16 word bits go to LDS (wm16[c],
// PACK: the pre-joiner bits to wb16[c]) and lane L reads back its contiguous
// 64-byte segment (chunks 4 L .. 4 L + 3) as one u64: no strided ds_read_b128
// of the text (the round-3 classify's bank conflicts) and no work on the rows
// past the document.  Neighbour bytes across chunks by wave shuffles, across
// rows from the staged text (lanes 0 / 63).
// UNI (round 5, documents the ASCII pass flagged): bytes >= 0x80 read as
// letters — right once uni_simple_span has passed the document (every
// non-ASCII char a well-formed ALetter that is its own lower case); the SWAR
// tests run on the low 7 bits with the high bytes masked out (their adds
// would carry into the next byte).
__device__ __forceinline__ uint32_t ld_byte_u(uint32_t c) { return c >= 0x80u ? 0x80u : ld_byte(c); }

template <bool PACK, bool UNI = false>
__device__ __forceinline__ uint64_t regs_word_mask(const uint4 *v, uint32_t nrows, const uint8_t *text,
                                                   uint16_t *wm16, uint16_t *wb16, uint32_t lane, bool *bad,
                                                   bool *under, uint64_t *wbase, bool *upper) {
  uint32_t badacc = 0, U = 0, us = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if ((uint32_t)k >= nrows) break;                          // wave-uniform
    const uint32_t xr[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
    uint32_t x[4], hb[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      hb[i] = UNI ? xr[i] & 0x80808080u : 0u;
      x[i] = UNI ? xr[i] & 0x7F7F7F7Fu : xr[i];
    }
    uint32_t LD[4], P = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t D = UNI ? swar_digit(x[i]) & ~hb[i] : swar_digit(x[i]);
      const uint32_t La = UNI ? swar_letter(x[i]) & ~hb[i] : swar_letter(x[i]);
      const uint32_t Lt = La | hb[i];
      LD[i] = Lt | (D >> 1);
      U |= La & ~(x[i] << 2);
      badacc |= xr[i];
      P |= (x[i] + 0x59595959u) & ~(x[i] + 0x44444444u) & ~D & ~hb[i];
    }
    uint32_t ldp = (uint32_t)__shfl_up((int)LD[3], 1, 64);
    uint32_t ldn = (uint32_t)__shfl_down((int)LD[0], 1, 64);
    if (lane == 0) ldp = k ? (UNI ? ld_byte_u(text[1024 * k - 1]) : ld_byte(text[1024 * k - 1])) << 24 : 0u;
    if (lane == 63) ldn = k < 3 ? (UNI ? ld_byte_u(text[1024 * k + 1024]) : ld_byte(text[1024 * k + 1024])) : 0u;
    const bool mids = __any((P & 0x80808080u) != 0);
    uint32_t W = 0, WB = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t u = UNI ? swar_eq(x[i], 0x5F5F5F5Fu) & ~hb[i] : swar_eq(x[i], 0x5F5F5F5Fu);
      us |= u;
      uint32_t c = LD[i] | (LD[i] << 1) | u;
      if (PACK) WB |= swar_nib(c & 0x80808080u) << (4 * i);
      if (mids) {
        const uint32_t prev4 = i ? LD[i - 1] : ldp;
        const uint32_t next4 = i < 3 ? LD[i + 1] : ldn;
        const uint32_t pf = __builtin_amdgcn_alignbyte(LD[i], prev4, 3);
        const uint32_t nf = __builtin_amdgcn_alignbyte(next4, LD[i], 1);
        const uint32_t both = pf & nf;
        const uint32_t dq = swar_eq(x[i], 0x2E2E2E2Eu) | swar_eq(x[i], 0x27272727u);
        const uint32_t ml = (dq | swar_eq(x[i], 0x3A3A3A3Au)) & ~hb[i];
        const uint32_t mn = (dq | swar_eq(x[i], 0x2C2C2C2Cu) | swar_eq(x[i], 0x3B3B3B3Bu)) & ~hb[i];
        c |= (ml & both) | (mn & (both << 1));
      }
      W |= swar_nib(c & 0x80808080u) << (4 * i);
    }
    wm16[64 * k + lane] = (uint16_t)W;
    if (PACK) wb16[64 * k + lane] = (uint16_t)WB;
  }
  asm volatile("" ::: "memory");
  *upper = __any(U != 0);
  *bad = __any((badacc & 0x80808080u) != 0);
  *under = __any(us != 0);
  const bool in = (lane >> 4) < nrows;
  if (PACK) *wbase = in ? reinterpret_cast<const uint64_t *>(wb16)[lane] : 0ull;
  return in ? reinterpret_cast<const uint64_t *>(wm16)[lane] : 0ull;
}

// Folded table key of a token of 9..255 bytes at tp (see above); *h slot hash.
// UNI: any length; bit 8 (free outside packs) set when the token holds a
// non-ASCII byte (its dictionary key then comes from the Unicode key builder).
constexpr uint64_t kFoldUni = 1ull << 8;
template <bool UNI = false>
__device__ __noinline__ uint64_t fold_key(const uint8_t *text, uint32_t tp, uint32_t n, uint32_t *h, bool *valid) {
  const uint32_t *tw = reinterpret_cast<const uint32_t *>(text);
  const uint32_t a0 = tp >> 2, o = tp & 3;
  uint32_t h1 = 0x243F6A88u ^ n, h2 = 0x85A308D3u + n, nu = 0, hib = 0;
  uint32_t prev = tw[a0];
  for (uint32_t i = 0; 4 * i < n; i++) {
    const uint32_t nx = tw[a0 + i + 1];
    const uint32_t k = keep_bytes(n, i);
    const uint32_t t = __builtin_amdgcn_alignbyte(nx, prev, o) & k;
    prev = nx;
    if (UNI) hib |= t;
    nu |= (t ^ 0x5F5F5F5Fu) & k;
    const uint32_t l = lower4(t);
    h1 = (h1 ^ l) * 0x9E3779B1u; h1 = __builtin_rotateleft32(h1, 13);
    h2 = (h2 ^ l) * 0x85EBCA77u; h2 = __builtin_rotateleft32(h2, 17);
  }
  h1 ^= h1 >> 16; h1 *= 0x2C1B3C6Du; h1 ^= h1 >> 13;
  h2 ^= h2 >> 16; h2 *= 0x297A2D39u; h2 ^= h2 >> 13;
  *h = h2;
  *valid = nu != 0;
  return kFoldBit | (uint64_t)n | ((uint64_t)tp << 13) | ((uint64_t)h1 << 26) | (((uint64_t)(h1 ^ h2) & 31ull) << 58) |
         ((hib & 0x80808080u) ? kFoldUni : 0ull);
}

// Lower-cased byte equality of the n-byte spans at p1 and p2.
__device__ __noinline__ bool span_same(const uint8_t *text, uint32_t p1, uint32_t p2, uint32_t n) {
  const uint32_t *tw = reinterpret_cast<const uint32_t *>(text);
  const uint32_t a1 = p1 >> 2, o1 = p1 & 3, a2 = p2 >> 2, o2 = p2 & 3;
  for (uint32_t i = 0; 4 * i < n; i++) {
    const uint32_t x = __builtin_amdgcn_alignbyte(tw[a1 + i + 1], tw[a1 + i], o1);
    const uint32_t y = __builtin_amdgcn_alignbyte(tw[a2 + i + 1], tw[a2 + i], o2);
    if ((lower4(x) ^ lower4(y)) & keep_bytes(n, i)) return false;
  }
  return true;
}

// Does a CAS that returned `old` resolve the token keyed `tk`?  (claimed the
// empty slot, or found the same term)
__device__ __forceinline__ bool table_hit(const uint8_t *text, uint64_t old, uint64_t tk) {
  if (old == 0 || old == tk) return true;
  if ((tk & old & kFoldBit) && ((old ^ tk) & ~kFoldPosMask) == 0)
    return span_same(text, (uint32_t)(old >> 13) & 0x1FFFu, (uint32_t)(tk >> 13) & 0x1FFFu, (uint32_t)tk & 0xFFu);
  return false;
}

// One bucket probe of a short key (dictionary lo array, 2-slot bucket at s & ~1,
// slots >= s considered).  Returns the found slot, or kLookupPending with
// *claim = slot to claim (empty) or kInvalidSlot (advance to the next bucket).
__device__ __forceinline__ uint32_t bucket_probe(ulonglong2 e, uint32_t s, uint64_t lo, uint32_t *claim) {
  const bool odd = (s & 1u) != 0;
  const uint64_t v0 = odd ? e.y : e.x;
  const bool f0 = v0 == lo, z0 = v0 == 0;
  const bool f1 = !odd & (e.y == lo), z1 = !odd & (e.y == 0);
  const bool hit = f0 | (!z0 & f1);
  const bool cl = z0 | (!f0 & !f1 & z1);
  *claim = cl ? (z0 ? s : s + 1) : kInvalidSlot;
  return hit ? (f0 ? s : s + 1) : kLookupPending;
}

// The same over the aligned 4-slot group of s (two 16 B loads, e0 = slots
// 0-1, e1 = slots 2-3; slots >= s considered in probe order): a key displaced
// by up to three slots from its home is found in the first round.
__device__ __forceinline__ uint32_t group_probe(ulonglong2 e0, ulonglong2 e1, uint32_t s, uint64_t lo,
                                                uint32_t *claim) {
  const uint32_t g0 = s & ~3u, off = s & 3u;
  const uint64_t v[4] = {e0.x, e0.y, e1.x, e1.y};
  uint32_t hit = kLookupPending, cl = kInvalidSlot;
#pragma unroll
  for (int i = 3; i >= 0; i--) {                           // the lowest slot >= s decides
    if ((uint32_t)i >= off) {
      const bool f = v[i] == lo, z = v[i] == 0;
      hit = f ? g0 + i : (z ? kLookupPending : hit);
      cl = f ? kInvalidSlot : (z ? g0 + i : cl);
    }
  }
  *claim = cl;
  return hit;
}

// The same over the aligned N-slot window of s (N / 2 16 B loads in e[]):
// the retry queue's probes, so a key displaced further than its first
// round's bucket costs one more dependent round trip, not one per bucket.
template <int N>
__device__ __forceinline__ uint32_t window_probe(const ulonglong2 *e, uint32_t s, uint64_t lo, uint32_t *claim) {
  const uint32_t g0 = s & ~(uint32_t)(N - 1), off = s & (uint32_t)(N - 1);
  uint32_t hit = kLookupPending, cl = kInvalidSlot;
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {                       // the lowest slot >= s decides
    if ((uint32_t)i >= off) {
      const uint64_t v = (i & 1) ? e[i >> 1].y : e[i >> 1].x;
      const bool f = v == lo, z = v == 0;
      hit = f ? g0 + i : (z ? kLookupPending : hit);
      cl = f ? kInvalidSlot : (z ? g0 + i : cl);
    }
  }
  *claim = cl;
  return hit;
}
#ifndef TFIDF_QWIN_G4
#define TFIDF_QWIN_G4 16
#endif
#ifndef TFIDF_QWIN_G2
#define TFIDF_QWIN_G2 2
#endif
// slots per retry-queue probe: one 128 B line (16) for dictionaries outside
// L2 (G4; cfg 5 tokenize 11.95 -> 11.27 ms, 8 slots 11.55), the 2-slot bucket
// for L2-resident ones (8 there: cfg 2 6.78 -> 6.87 ms, 4: 6.81)
template <bool G4>
constexpr int queue_win() { return G4 ? TFIDF_QWIN_G4 : TFIDF_QWIN_G2; }

// Claim slot cs for short key lo (CAS on lo, then publish hi).  Returns the
// slot if it now holds lo, else kLookupPending with *s advanced past cs.
__device__ __forceinline__ uint32_t dict_claim_short(uint64_t *dict, uint32_t mask, uint32_t cs, uint64_t lo,
                                                     uint32_t *s) {
  const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long *>(dict + cs), 0ull,
                                           (unsigned long long)lo);
  if (old == 0) __hip_atomic_store(dict + (size_t)mask + 1 + cs, kKeyValid, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  if (old == 0 || old == lo) return cs;
  *s = (cs + 1) & mask;
  return kLookupPending;
}

// 16-bit field f of a packed 8-field value (two fields per word)
__device__ __forceinline__ uint32_t field8(const uint32_t *w, uint32_t f) {
  const uint32_t h = f >> 1;
  const uint32_t v = h == 0 ? w[0] : (h == 1 ? w[1] : (h == 2 ? w[2] : w[3]));
  return (v >> (16 * (f & 1))) & 0xFFFFu;
}
__device__ __forceinline__ void field8_add(uint32_t *w, uint32_t f, uint32_t inc16) {
  const uint32_t h = f >> 1, inc = inc16 << (16 * (f & 1));
  w[0] += h == 0 ? inc : 0u;
  w[1] += h == 1 ? inc : 0u;
  w[2] += h == 2 ? inc : 0u;
  w[3] += h == 3 ? inc : 0u;
}

__device__ __forceinline__ uint4 gload16(const void *ptr) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(1))) const uint32_t gu32;
  gu32 *g = (gu32 *)ptr;
  // streamed once: non-temporal, so the dictionary keeps its L2 lines
  // (with the non-temporal CSR stores: tokenize 8.32 -> 8.27 ms at cfg 2)
  return make_uint4(__builtin_nontemporal_load(g), __builtin_nontemporal_load(g + 1), __builtin_nontemporal_load(g + 2),
                    __builtin_nontemporal_load(g + 3));
#else
  return *reinterpret_cast<const uint4 *>(ptr);
#endif
}

// One unit of the wave path: d = first (committed) document, src = its
// staged source, [s0, s0 + L) = the window's corpus bytes.  PACK: np documents
// d .. d + np - 1 with sources src .. src + np - 1; lane j <= np holds pofs =
// the corpus offset of document j (lane np: the end); ok = the sources are
// contiguous and no document is empty (the boundaries are distinct).
struct DocMeta {
  uint64_t d, s0, L, src, pofs;
  uint32_t shift, np;
  bool ok;
};

template <bool PACK>
__device__ __forceinline__ DocMeta unit_meta(const BuildParams &p, uint64_t u, uint32_t lane) {
  DocMeta m;
  if (!PACK) {
    m.d = TFIDF_COLD(doc_list) ? TFIDF_COLD(doc_list)[u] : u;
    m.src = TFIDF_COLD(live_map) ? TFIDF_COLD(live_map)[m.d] : m.d;
    m.s0 = p.offsets[m.src];
    m.L = p.offsets[m.src + 1] - m.s0;
    m.pofs = 0;
    m.np = 1;
    m.ok = true;
  } else {
    m.d = u * p.pack;
    const uint32_t np = (uint32_t)min((uint64_t)p.pack, p.n_docs - m.d);
    const uint32_t j = lane < np ? lane : np - 1;
    // lane j < np: source of document d + j; lanes >= np: one past the last source
    const uint64_t sj = (TFIDF_COLD(live_map) ? (uint64_t)TFIDF_COLD(live_map)[m.d + j] : m.d + j) + (lane < np ? 0u : 1u);
    m.src = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(sj >> 32), 0) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sj, 0);
    const bool contig = __all(lane > np || sj == m.src + lane);
    m.pofs = p.offsets[sj];
    const uint64_t nxt = ((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)(m.pofs >> 32), 1, 64) << 32) |
                         (uint32_t)__shfl_down((int)(uint32_t)m.pofs, 1, 64);
    const bool nonempty = __all(lane >= np || nxt > m.pofs);
    m.s0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m.pofs >> 32), 0) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m.pofs, 0);
    const uint64_t end = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m.pofs >> 32), (int)np) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m.pofs, (int)np);
    m.L = end - m.s0;
    m.np = np;
    m.ok = contig && nonempty;
  }
  m.shift = (uint32_t)(reinterpret_cast<uintptr_t>(p.text + m.s0) & 15);
  return m;
}

__device__ __forceinline__ bool fits_wave(const DocMeta &m) { return m.ok && m.shift + m.L <= kWaveWindow; }

// PACK: documents d .. d + np - 1 go to the single-document pass.
__device__ __forceinline__ void defer_pack(const BuildParams &p, uint64_t d, uint32_t np, uint32_t lane) {
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(TFIDF_COLD(retry_count), np);
  base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
  if (lane < np) TFIDF_COLD(retry_list)[base + lane] = (uint32_t)(d + lane);
}

__device__ __forceinline__ void prefetch_wave(const BuildParams &p, const DocMeta &m, uint32_t lane, uint4 *v) {
  if (!fits_wave(m)) return;
  const uint32_t nchunks = (uint32_t)((m.shift + m.L + 15) >> 4);
  const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(p.text + m.s0) & ~(uintptr_t)15);
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (lane + 64 * k < nchunks) v[k] = gload16(src + lane + 64 * k);
}

// bytes of the dword at window byte q that lie in [lo, hi)
__device__ __forceinline__ uint32_t keep_range(uint32_t q, uint32_t lo, uint32_t hi) {
  const uint32_t a = q >= lo ? 0xFFFFFFFFu : (lo - q >= 4 ? 0u : (0xFFFFFFFFu << (8 * (lo - q))));
  const uint32_t b = q + 4 <= hi ? 0xFFFFFFFFu : (hi <= q ? 0u : (0xFFFFFFFFu >> (8 * (q + 4 - hi))));
  return a & b;
}

__device__ __forceinline__ void clear_table(WaveSmem &sm, uint32_t lane) {
  uint4 *kw = reinterpret_cast<uint4 *>(sm.key);
  uint4 *cw = reinterpret_cast<uint4 *>(sm.cnt);
#pragma unroll
  for (int q = 0; q < (int)(kWaveSlots * 8 / 16 / 64); q++) kw[lane + 64 * q] = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int q = 0; q < (int)(kWaveSlots * 2 / 16 / 64); q++) cw[lane + 64 * q] = make_uint4(0, 0, 0, 0);
}

// ---- histogram, lane-mask form (round 3).  Per-token state that is a
// yes/no per lane (in range, pending, hit) stays in wave lane masks (SGPRs):
// the probe bookkeeping and the token / distinct-term counts are scalar
// instructions, and the conditional LDS atomics run under EXEC instead of
// being aimed at no-op slots.  Keys are cut out of the staged text with one
// v_perm_b32 per key dword, whose selector (from a small LDS table indexed by
// token length and start & 3) both aligns the bytes and zeroes those past the
// token's end.  Slot hash: one full-rate 24-bit multiply.
//
// Selector table (in the wave's former no-op area): entry 4 n + o, n = 0..8
// bytes, o = start & 3: {sel0, sel1}; key dword 0 = perm(dw1, dw0, sel0),
// dword 1 = perm(dw2, dw1, sel1) where dw0..2 are the text dwords from
// start & ~3; selector byte 12 yields 0x00.
constexpr uint32_t kSelEntries = 36;
__device__ __forceinline__ void init_sel_table(uint2 *tab, uint32_t lane) {
  if (lane < kSelEntries) {
    const uint32_t n = lane >> 2, o = lane & 3;
    uint32_t s0 = 0, s1 = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
      s0 |= (i < n ? o + i : 12u) << (8 * i);
      s1 |= (i + 4 < n ? o + i : 12u) << (8 * i);
    }
    tab[lane] = make_uint2(s0, s1);
  }
}
__device__ __forceinline__ uint32_t table_slot(uint32_t l0, uint32_t l1) {
  const uint32_t x = l0 ^ __builtin_amdgcn_alignbit(l1, l1, 16);
  return (uint32_t)__umul24(x ^ (x >> 11), 0x2C1B3Du) >> (32 - kWaveSlotBits);
}
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Wave lane masks as per-lane predicates: the SGPR mask is the VCC operand
// of the consuming instruction (no VALU).
__device__ __forceinline__ bool lane_in(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }

// One probe of up to J tokens per lane, the pending ones masked by pm[j]
// (wave lane masks): CAS on the slot (a lane with nothing to probe aims at a
// selector-table entry, never 0, so its compare-with-0 never writes), count
// the hits, retire them from pm, advance the others one slot.  Returns the
// tokens still pending.
template <int J, bool FOLD, class SM>
__device__ __forceinline__ uint32_t probe_round(SM &sm, uint32_t lane, const uint64_t *tk, uint32_t *slot,
                                                uint64_t *pm, uint32_t &claims) {
  unsigned long long *idle = reinterpret_cast<unsigned long long *>(&sm.sel[lane & 31]);
  uint32_t *idle32 = reinterpret_cast<uint32_t *>(idle);
  uint64_t old[J];
#pragma unroll
  for (int j = 0; j < J; j++)
    old[j] = atomicCAS(lane_in(pm[j]) ? reinterpret_cast<unsigned long long *>(&sm.key[slot[j]]) : idle, 0ull,
                       (unsigned long long)tk[j]);
  __builtin_amdgcn_sched_barrier(0);     // every CAS issued before the first result is waited on
  uint32_t P = 0;
#pragma unroll
  for (int j = 0; j < J; j++) {
    const uint64_t zm = __ballot(old[j] == 0) & pm[j];
    uint64_t hm = (__ballot(old[j] == tk[j]) & pm[j]) | zm;
    // same length and folded hash, other position: compare the bytes (only
    // while a pending lane holds a folded key: one compare + mask test per
    // round otherwise)
    if (FOLD && (__ballot((int32_t)(uint32_t)(tk[j] >> 32) < 0) & pm[j] & ~hm)) {
      const uint64_t fm = __ballot((((old[j] & tk[j]) >> 63) != 0) & (((old[j] ^ tk[j]) & ~kFoldPosMask) == 0)) &
                          pm[j] & ~hm;
      if (fm) {
        bool same = false;
        if (lane_in(fm))
          same = span_same(sm.text, (uint32_t)(old[j] >> 13) & 0x1FFFu, (uint32_t)(tk[j] >> 13) & 0x1FFFu,
                           (uint32_t)tk[j] & 0xFFu);
        hm |= __ballot(same) & fm;
      }
    }
    const bool hit = lane_in(hm);
    atomicAdd(hit ? &sm.cnt[slot[j] >> 1] : idle32, hit ? 1u << (16 * (slot[j] & 1)) : 0u);
    claims += (uint32_t)__popcll(zm);
    pm[j] &= ~hm;
    slot[j] = (slot[j] + (lane_in(pm[j]) ? 1u : 0u)) & (kWaveSlots - 1);
    P += (uint32_t)__popcll(pm[j]);
  }
  return P;
}

// One batch of 64 K tokens [tb, tb + 64 K) of the list (entries past ntok
// are ignored).  claims / toks: wave-uniform running counts of distinct
// terms / counted tokens.
// UNI: a token holding a byte >= 0x80 takes a folded key whatever its length
// (fold_key / span_same lower-case the ASCII bytes only; a UNI document's
// non-ASCII chars are their own lower case, and lower4's byte adds leave the
// bytes of well-formed UTF-8 unchanged).
template <int K, bool FOLD, bool PACK, bool UNI = false>
__device__ __forceinline__ void hist2(WaveSmem &sm, uint32_t lane, uint32_t tb, uint32_t ntok, bool under, bool upper,
                                      uint32_t &claims, uint32_t &toks, bool &overflow) {
  const uint32_t *tw = reinterpret_cast<const uint32_t *>(sm.text);
  const uint32_t left = ntok - tb;                       // wave-uniform
  uint32_t ent[K], dw[K][3];
  uint2 sl[K];
#pragma unroll
  for (int k = 0; k < K; k++) ent[k] = sm.list[tb + lane + 64 * k];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t tp = ent[k] & kSpanMask, n = ((ent[k] >> 16) & kSpanMask) - tp;
    const uint32_t a0 = tp >> 2;
    dw[k][0] = tw[a0]; dw[k][1] = tw[a0 + 1]; dw[k][2] = tw[a0 + 2];
    sl[k] = sm.sel[(min(n, 8u) << 2) | (tp & 3u)];
  }
  uint64_t tkey[K], pm[K];
  uint32_t slot[K];
  uint32_t t0[K], t1[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    t0[k] = __builtin_amdgcn_perm(dw[k][1], dw[k][0], sl[k].x);
    t1[k] = __builtin_amdgcn_perm(dw[k][2], dw[k][1], sl[k].y);
  }
  if (upper) {
#pragma unroll
    for (int k = 0; k < K; k++) { t0[k] = lower4(t0[k]); t1[k] = lower4(t1[k]); }
  }
  uint64_t lm = 0;                                       // FOLD: lanes with a token of 9+ bytes, per k (bit k)
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint32_t tp = ent[k] & kSpanMask, n = ((ent[k] >> 16) & kSpanMask) - tp;
    const bool in = lane + 64u * k < left;
    bool valid = true;
    if (FOLD && under)   // a span of '_' only is not a token
      valid = (t0[k] != __builtin_amdgcn_perm(0x5F5F5F5Fu, 0x5F5F5F5Fu, sl[k].x)) |
              (t1[k] != __builtin_amdgcn_perm(0x5F5F5F5Fu, 0x5F5F5F5Fu, sl[k].y));
    const uint32_t l0 = t0[k] | (PACK ? pack_tag(span_doc(ent[k])) : 0u);
    tkey[k] = (uint64_t)l0 | ((uint64_t)t1[k] << 32);
    slot[k] = table_slot(l0, t1[k]);
    // UNI: an 8-byte token holding a non-ASCII byte takes a folded key (its byte
    // 7 may have bit 63's place; marked in the entry's spare bit 31 for the fold
    // block); shorter ones keep their bytes as the table key (bit 63 clear:
    // exact identity, their dictionary key derived from it).  (A document with
    // an 8-byte token runs the folded histogram: the span loop counts them long.)
    const bool hh = UNI && n == 8 && ((t0[k] | t1[k]) & 0x80808080u) != 0;
    if (UNI) ent[k] |= hh ? 0x80000000u : 0u;
    pm[k] = __ballot(in & (n <= 8) & valid & !hh);
    if (FOLD) lm |= (uint64_t)(__ballot(in & ((n > 8) | hh)) != 0) << k;
  }
  if (FOLD && lm) {                                      // tokens of 9..255 bytes: folded keys
    bool toolong = false;
#pragma unroll
    for (int k = 0; k < K; k++) {
      if ((lm >> k) & 1u) {
        const uint32_t e = ent[k];
        const uint32_t tp = e & kSpanMask, n = ((e >> 16) & kSpanMask) - tp;
        bool ok = false;
        if (lane + 64u * k < left && (n > 8 || (UNI && (e >> 31) != 0 && n == 8))) {
          if (n > kMaxTokenLen) {
            toolong = true;
          } else {
            uint32_t h;
            tkey[k] = fold_key<UNI>(sm.text, tp, n, &h, &ok);
            if (PACK) {
              tkey[k] |= (uint64_t)span_doc(e) << 8;
              h ^= span_doc(e) * 0x9E3779B1u;
            }
            slot[k] = h >> (32 - kWaveSlotBits);
          }
        }
        pm[k] |= __ballot(ok);
      }
    }
    if (__any(toolong)) { overflow = true; return; }     // > 255 chars: the long path cuts it
  }
  uint32_t P = 0;
#pragma unroll
  for (int k = 0; k < K; k++) P += (uint32_t)__popcll(pm[k]);
  toks += P;
  // probe rounds over every token while many remain (the first resolves ~90 %)
  for (uint32_t round = 0; P > kWaveQueue; round++) {
    if (round >= kWaveSlots) { overflow = true; return; }
    P = probe_round<K, FOLD>(sm, lane, tkey, slot, pm, claims);
  }
  if (P == 0) return;
  // the rest (<= 128): compacted into a queue, one or two per lane, probed to the end
  {
    uint32_t at = 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      if (pm[k]) {
        if (lane_in(pm[k])) {
          const uint32_t q = at + lanes_below(pm[k]);
          sm.qkey[q] = tkey[k];
          sm.qslot[q] = (uint16_t)slot[k];
        }
        at += (uint32_t)__popcll(pm[k]);
      }
    }
  }
  asm volatile("" ::: "memory");
  uint64_t qk[2];
  uint32_t qs[2];
  uint64_t qm[2];
#pragma unroll
  for (int i = 0; i < 2; i++) {
    const bool qp = lane + 64u * i < P;
    qk[i] = qp ? sm.qkey[lane + 64 * i] : 0ull;
    qs[i] = qp ? sm.qslot[lane + 64 * i] : 0u;
    qm[i] = __ballot(qp);
  }
  for (uint32_t it = 0;; it++) {
    if (it >= kWaveSlots) { overflow = true; return; }
    const uint32_t left_q = P > 64 ? probe_round<2, FOLD>(sm, lane, qk, qs, qm, claims)
                                   : probe_round<1, FOLD>(sm, lane, qk, qs, qm, claims);
    if (left_q == 0) return;
  }
}

// Dictionary slots of the document's distinct terms (table entries listed in
// slots[0, nu)): lane l resolves terms l + 64k (k < kWaveK) -> g[k], with
// their counts tf[k] (and, PACK, the pack-local document tdoc[k]; per-document
// lengths / term counts accumulated into pk_len / pk_nu).  Short keys by
// bucket probes with all of a lane's loads in flight, unresolved ones through
// a one-per-lane retry queue; folded (> 8 byte) keys one per lane at a time.
// UNI: dictionary slot of a folded term (128-bit key lo / hi, occurrence
// mine) with its identity check, in fewer dependent round trips than
// dict_find_or_insert + verify_lds: each probe loads the bucket's keys lo, hi
// AND reference words together, so a term found in its home bucket costs one
// round trip plus one for the spelling check.  Returns slot | status << 32:
// 0 nothing to check (claimed, exact key, or the reference spelled the same),
// 1 found with no reference visible yet (the caller defers through
// dict_verify), 2 another term under the key (a collision); slot
// kInvalidSlot: dictionary full.
__device__ __noinline__ uint64_t uni_find_verify(uint64_t *dict, uint32_t mask, uint64_t lo, uint64_t hi,
                                                 uint64_t mine, const uint8_t *text, const uint8_t *wtext, uint32_t tp) {
  uint64_t *dlo = dict, *dhi = dict + (size_t)mask + 1, *dref = dict + 2 * ((size_t)mask + 1);
  uint32_t s = dict_home(dict_hash(lo, hi), mask) & ~1u;     // probing starts at the bucket (dict_lookup_multi)
  uint32_t slot = kInvalidSlot;
  uint64_t r = 0;
  for (uint32_t it = 0; it < mask + 1 + 4096 && slot == kInvalidSlot; it++) {
    const uint32_t b = s & ~1u;
    const ulonglong2 el = *reinterpret_cast<const ulonglong2 *>(dlo + b);
    const ulonglong2 eh = *reinterpret_cast<const ulonglong2 *>(dhi + b);
    const ulonglong2 er = *reinterpret_cast<const ulonglong2 *>(dref + b);
    uint32_t next = (b + 2) & mask;
    for (uint32_t q = s & 1u; q < 2 && slot == kInvalidSlot; q++) {
      const uint32_t js = b + q;
      uint64_t v = q ? el.y : el.x;
      if (v == 0) {                                        // empty (or stale): claim
        v = atomicCAS(reinterpret_cast<unsigned long long *>(dlo + js), 0ull, (unsigned long long)lo);
        if (v == 0) {
          if (lo & kLoHashed) __hip_atomic_store(dref + js, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(dhi + js, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return js;                                       // claimed: this occurrence is the reference
        }
      }
      if (v != lo) continue;
      uint64_t h = q ? eh.y : eh.x;
      for (uint32_t w = 0; h == 0 && w < (1u << 20); w++)   // claimed, hi not published yet
        h = __hip_atomic_load(dhi + js, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (h == hi) {
        slot = js;
        r = q ? er.y : er.x;
      } else if (h == 0) {
        next = js;                                         // (bounded wait over) probe it again
        break;
      }
    }
    s = next;
  }
  if (slot == kInvalidSlot || !(lo & kLoHashed)) return slot;
  if (r == 0) r = __hip_atomic_load(dref + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (r == mine) return slot;
  if (r == 0) return slot | (1ull << 32);
  const uint32_t n = dict_ref_len(mine);
  if (n == dict_ref_len(r) && n <= 32) {
    const uint64_t off = dict_ref_off(r);
    const uint32_t o = (uint32_t)(off & 3u), lo4 = tp & 3u;
    const uint32_t *g = reinterpret_cast<const uint32_t *>(text + (off & ~3ull));
    const uint32_t *l = reinterpret_cast<const uint32_t *>(wtext + (tp & ~3u));
    uint32_t gw[9], lw[9];
#pragma unroll
    for (int j = 0; j < 9; j++) {
      gw[j] = 4u * j < o + n ? g[j] : 0u;
      lw[j] = 4u * j < lo4 + n ? l[j] : 0u;
    }
    uint32_t diff = 0;
#pragma unroll
    for (int j = 0; j < 8; j++)
      diff |= (__builtin_amdgcn_alignbyte(gw[j + 1], gw[j], o) ^ __builtin_amdgcn_alignbyte(lw[j + 1], lw[j], lo4)) &
              keep_bytes(n, j);
    if (diff == 0) return slot;
  }
  const bool same = uc_same_term(text + dict_ref_off(r), dict_ref_len(r), text + dict_ref_off(mine), n);
  return slot | (same ? 0ull : (2ull << 32));
}

// UNI: folded terms keyed by the Unicode key builder (lower-cased code
// points; the same key the Unicode and long paths give the term).
// UNI: dictionary key of a short table key holding a non-ASCII byte (the
// token's lower-cased bytes, <= 7 of them: an exact key, no identity check,
// so no occurrence is needed).
__device__ __forceinline__ void uni_key_from_short(uint64_t key, uint64_t *lo, uint64_t *hi) {
  // KeyBuilder over the key's bytes, in closed form: a non-ASCII key of <= 7
  // bytes takes KeyBuilder::finish's exact branch (w0 = the bytes, w1 = 0).
  // (Inline: the call it replaces saved the resolve phase's live registers
  // to scratch around every folded term.)
  const uint64_t n = key ? (uint64_t)((71 - __builtin_clzll(key)) >> 3) : 0ull;
  const uint64_t r = (key >> 63) | (n << 49);
  *lo = kLoLong | kLoUniExact | (r & ((1ull << 47) - 1)) | ((r >> 47) << 48);
  *hi = (key & ~kKeyValid) | kKeyValid;
}

// The document passed uni_simple_char, so its non-ASCII chars are their own
// lower case: the key builder's bytes are the token's with ASCII lower-cased
// (what uc_token_key would push, without decoding or the case tables).
__device__ __noinline__ void uni_dict_key(const uint8_t *text, uint32_t tp, uint32_t n, uint64_t *lo, uint64_t *hi,
                                          uint64_t seed) {
  KeyBuilder kb;
  for (uint32_t j = tp; j < tp + n; j++) kb.push(ascii_lower(text[j]));
  kb.finish(lo, hi, seed);
}

template <bool PACK, bool G4, bool UNI = false>
__device__ __forceinline__ void resolve_terms(WaveSmem &sm, const BuildParams &p, uint32_t lane, uint32_t nu,
                                              uint32_t doc, uint32_t *g, uint32_t *tf, uint32_t *tdoc,
                                              uint32_t &actm, uint32_t *pk_len, uint32_t *pk_nu, uint64_t wbase,
                                              uint32_t wlen = 0) {
  const uint32_t dmask = p.cap_mask;
  const uint16_t *slots = reinterpret_cast<const uint16_t *>(sm.list);
  if (PACK && lane < kPackMax) { pk_len[lane] = 0; pk_nu[lane] = 0; }
  {
    uint64_t lo[kWaveK];
    uint32_t ps[kWaveK];
    uint32_t foldm = 0;
#pragma unroll
    for (int k = 0; k < (int)kWaveK; k++) {
      lo[k] = 0;
      tf[k] = 0;
      g[k] = kInvalidSlot;
      ps[k] = 0;
      {
        const uint32_t idx = lane + 64 * k;
        const bool in = idx < nu;
        const uint32_t s = slots[in ? idx : 0u] & (kWaveSlots - 1);
        const uint64_t key = sm.key[s];
        tf[k] = (sm.cnt[s >> 1] >> (16 * (s & 1))) & 0xFFFFu;
        // UNI: a short table key holding a non-ASCII byte is not its dictionary key
        const bool f = in & (((key & kFoldBit) != 0) | (UNI && (key & 0x8080808080808080ull) != 0));
        const bool sh = in & !f;
        tdoc[k] = PACK ? key_doc(key) : 0u;
        if (PACK && in) { atomicAdd(&pk_len[tdoc[k]], tf[k]); atomicAdd(&pk_nu[tdoc[k]], 1u); }
        lo[k] = sh ? (PACK ? key & ~kPackTagMask : key) : 0ull;
        foldm |= (uint32_t)f << k;
        actm |= (uint32_t)in << k;
        ps[k] = dict_home(dict_hash_short(lo[k]), dmask) & ~1u;
        g[k] = sh ? kLookupPending : g[k];
      }
    }
    // folded (> 8 byte) terms: exact 128-bit keys, one lookup per lane at a time
    while (__any(foldm != 0)) {
      uint64_t flo = 1, fhi = kKeyValid, mine = 0;
      uint32_t k = 0;
      const bool fa = foldm != 0;
      if (fa) {
        k = (uint32_t)__builtin_ctz(foldm);
        foldm &= foldm - 1;
        const uint64_t key = sm.key[slots[lane + 64 * k]];
        const uint32_t n = (uint32_t)key & 0xFFu, tp = (uint32_t)(key >> 13) & 0x1FFFu;
        bool valid;
        if (UNI && !(key & kFoldBit)) {                    // short non-ASCII term: exact key from its bytes
          uni_key_from_short(key, &flo, &fhi);
        } else {
          if (UNI && (key & kFoldUni)) uni_dict_key(sm.text, tp, n, &flo, &fhi, TFIDF_COLD(hash_seed));
          else token_key(sm.text, tp, tp + n, &flo, &fhi, &valid, TFIDF_COLD(hash_seed));
          mine = dict_ref_word(wbase + tp, n);
        }
      }
      uint32_t gg;
      if (UNI) {
        // exact keys (non-ASCII terms of <= kExactUniChars bytes: nearly all)
        // by the inline probe, all lanes together; hashed ones by the verifying
        // lookup (a call: the caller's live registers go to scratch around it —
        // cfg-2 prose with every term through it: 750 VMEM instructions per
        // document against the ASCII pass's 22, SQ counters)
        const bool hashed = fa && (flo & kLoHashed);
        gg = dict_find_or_insert(p.dict, dmask, flo, fhi, fa && !hashed);
        if (__any(hashed) && hashed) {
          const uint64_t res = uni_find_verify(p.dict, dmask, flo, fhi, mine, p.text, sm.text,
                                               (uint32_t)(sm.key[slots[lane + 64 * k]] >> 13) & 0x1FFFu);
          gg = (uint32_t)res;
          if ((res >> 32) == 1) dict_verify(p, gg, mine, doc);   // defers (or finds the reference published by now)
          else if ((res >> 32) == 2) set_build_err(TFIDF_COLD(err), kErrCollision, doc);
        }
      } else {
        bool cl;
        gg = dict_find_or_insert(p.dict, dmask, flo, fhi, fa, &mine, &cl);
        if (fa && (flo & kLoHashed) && !cl && gg != kInvalidSlot) dict_verify(p, gg, mine, doc);   // > 16 bytes
      }
#pragma unroll
      for (int kk = 0; kk < (int)kWaveK; kk++)
        if (fa && (uint32_t)kk == k) g[kk] = gg;
    }
    // short terms: bucket probes, all of a lane's loads in flight per round
    for (uint32_t round = 0;; round++) {
      uint32_t np = 0;
#pragma unroll
      for (int k = 0; k < (int)kWaveK; k++) np += g[k] == kLookupPending;
      const uint32_t pincl = wave_incl_add(np);
      const uint32_t P = (uint32_t)__builtin_amdgcn_readlane((int)pincl, 63);
      if (P == 0) break;
      if (round > 0 && P <= kDictQueue) {
        // retry queue in the (no longer needed) table: (lo, probe slot, term index)
        uint64_t *qlo = sm.key;
        uint2 *qmeta = reinterpret_cast<uint2 *>(sm.key + kDictQueue);
        uint32_t *res = reinterpret_cast<uint32_t *>(sm.key + 2 * kDictQueue);
        uint32_t at = pincl - np;
#pragma unroll
        for (int k = 0; k < (int)kWaveK; k++)
          if (g[k] == kLookupPending) { qlo[at] = lo[k]; qmeta[at] = make_uint2(ps[k], lane + 64 * k); at++; }
        asm volatile("" ::: "memory");
        const bool qa = lane < P;
        uint64_t ql = 0;
        uint2 qm = make_uint2(0, 0);
        if (qa) { ql = qlo[lane]; qm = qmeta[lane]; }
        uint32_t qs = qm.x, qg = qa ? kLookupPending : kInvalidSlot;
        for (uint32_t it = 0; it < dmask + 4096 && __any(qg == kLookupPending); it++) {
          if (qg == kLookupPending) {
            uint32_t cs;
            constexpr int QW = queue_win<G4>();
            ulonglong2 e[QW / 2];
            const ulonglong2 *wp = reinterpret_cast<const ulonglong2 *>(p.dict + (qs & ~(uint32_t)(QW - 1)));
#pragma unroll
            for (int i = 0; i < QW / 2; i++) e[i] = wp[i];
            qg = window_probe<QW>(e, qs, ql, &cs);
            if (qg == kLookupPending) {
              if (cs != kInvalidSlot) qg = dict_claim_short(p.dict, dmask, cs, ql, &qs);
              else qs = ((qs | (uint32_t)(QW - 1)) + 1u) & dmask;
            }
          }
        }
        if (qa) res[qm.y] = qg == kLookupPending ? kInvalidSlot : qg;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < (int)kWaveK; k++)
          if (g[k] == kLookupPending) g[k] = res[lane + 64 * k];
        break;
      }
      if (round > dmask) break;                          // table exhausted: capacity error below
      // G4 (dictionaries of >= 2^21 slots, outside L2): the aligned 4-slot group
      // of each probe (two 16 B loads) — fewer dependent rounds at high load
      // (cfg 5: tokenize 14.9 -> 12.9 ms); 2-slot buckets otherwise (the extra
      // registers spill: cfg 2 8.27 -> 8.77 ms)
      // G4: probes in two halves of kWaveK / 2 terms (two 16 B loads each) so
      // the group registers of all eight are not live at once.  (An 8-slot
      // window here, two terms at a time: 91 VGPRs spilled, cfg 5 tokenize
      // 13.1 -> 16.6 ms.)
      constexpr int KH = G4 ? (int)kWaveK / 2 : (int)kWaveK;
      uint32_t cs[kWaveK];
      bool anyclaim = false;
#pragma unroll
      for (int h = 0; h < (int)kWaveK / KH; h++) {
        ulonglong2 e0[KH], e1[G4 ? KH : 1];
#pragma unroll
        for (int i = 0; i < KH; i++) {
          const int k = h * KH + i;
          const uint32_t gs = g[k] == kLookupPending ? (ps[k] & (G4 ? ~3u : ~1u)) : 0u;
          e0[i] = *reinterpret_cast<const ulonglong2 *>(p.dict + gs);
          if constexpr (G4) e1[i] = *reinterpret_cast<const ulonglong2 *>(p.dict + gs + 2);
        }
#pragma unroll
        for (int i = 0; i < KH; i++) {
          const int k = h * KH + i;
          const bool pend = g[k] == kLookupPending;
          uint32_t c;
          uint32_t r;
          if constexpr (G4) r = group_probe(e0[i], e1[i], ps[k], lo[k], &c);
          else r = bucket_probe(e0[i], ps[k], lo[k], &c);
          cs[k] = pend ? c : kInvalidSlot;
          anyclaim |= pend & (c != kInvalidSlot);
          const bool adv = pend & (r == kLookupPending) & (c == kInvalidSlot);
          ps[k] = adv ? (((ps[k] | (G4 ? 3u : 1u)) + 1u) & dmask) : ps[k];
          g[k] = pend ? r : g[k];
        }
      }
      if (__any(anyclaim)) {
#pragma unroll
        for (int k = 0; k < (int)kWaveK; k++)
          if (cs[k] != kInvalidSlot) g[k] = dict_claim_short(p.dict, dmask, cs[k], lo[k], &ps[k]);
      }
    }
    bool caperr = false;
#pragma unroll
    for (int k = 0; k < (int)kWaveK; k++) {
      const bool e = (((actm >> k) & 1u) != 0) & ((g[k] == kInvalidSlot) | (g[k] == kLookupPending));
      caperr |= e;
      if (e) g[k] = 0;
    }
    if (caperr) set_err(TFIDF_COLD(err), kErrCapacity, doc);
  }
}

// A flag per document for k_tokenize_uwave (no shared counter: a list
// appended with one atomic per document serialised a corpus of non-ASCII
// documents on one address).  Not inlined: inline, the store changed the
// tokenizer's register allocation (247 VGPRs, cfg-2 tokenize +0.1 ms).  The
// array is an argument: a called function has no kernarg pointer (TFIDF_COLD).
__device__ __noinline__ void flag_unicode(uint32_t *flags, uint64_t d) { flags[d] = 1u; }

// UNI (rounds 5-6): can the wave rules take this document?  Every non-ASCII
// char must be well-formed UTF-8 (no orphan continuation bytes) and one of
//   * an ALetter that is its own lower case (é ü ñ ß α я …): UAX#29 treats it
//     as it treats an ASCII letter (ALetter is the ASCII letters' class), so
//     the ASCII rules with its bytes read as letters give the scanner's tokens;
//   * an ALetter whose lower case (JDK Character.toLowerCase) has the same
//     UTF-8 length and is such a letter (É Ö Ç Σ Я …): its bytes are
//     lowered in the staged window, so term identity is again decided by
//     ASCII lower-casing (round 6);
//   * a char of class Other (no-break space, curly double quotes, dashes,
//     ellipsis, guillemets …): a break on both sides, exactly as an ASCII
//     space — its bytes become spaces in the staged window (round 6);
//   * MidLetter / MidNum / MidNumLet (’ ‘ · …): kept in the window, read as
//     class Other by the classifier, and joined afterwards where UAX#29 joins
//     them (WB6/7: a letter on both sides; WB11/12: a digit on both sides;
//     lane_word_mask) (round 6).
// Anything else (Han, Katakana, Hebrew, combining marks, non-ASCII digits or
// ExtendNumLet, emoji, malformed bytes) stays flagged for k_tokenize_uwave.
// One char through the tables: its lead byte and the three after it in w
// (little-endian), avail = bytes of the window from the lead on; returns
// kind | byte length << 4 | (kPrUpper) the lower case's UTF-8 bytes << 8.
// (Bytes come in registers: a generic pointer into LDS would be flat loads,
// one dependent round trip per byte — 4.6 ms at cfg 2 with every document
// non-ASCII.)
enum : uint32_t { kPrNo = 0, kPrLetter, kPrUpper, kPrSep, kPrMidL, kPrMidN, kPrMidNL };
__device__ __noinline__ uint32_t uni_prose_char(uint32_t w, uint32_t avail) {
  const uint32_t b0 = w & 0xFFu, b1 = (w >> 8) & 0xFFu, b2 = (w >> 16) & 0xFFu, b3 = w >> 24;
  auto cont = [](uint32_t b, uint32_t lo, uint32_t hi) { return b >= lo && b <= hi; };
  uint32_t cp, len;
  if (b0 >= 0xC2u && b0 < 0xE0u && avail >= 2 && cont(b1, 0x80u, 0xBFu)) {
    cp = ((b0 & 0x1Fu) << 6) | (b1 & 0x3Fu);
    len = 2;
  } else if (b0 >= 0xE0u && b0 < 0xF0u && avail >= 3 && cont(b1, b0 == 0xE0u ? 0xA0u : 0x80u, b0 == 0xEDu ? 0x9Fu : 0xBFu) &&
             cont(b2, 0x80u, 0xBFu)) {
    cp = ((b0 & 0x0Fu) << 12) | ((b1 & 0x3Fu) << 6) | (b2 & 0x3Fu);
    len = 3;
  } else if (b0 >= 0xF0u && b0 < 0xF5u && avail >= 4 && cont(b1, b0 == 0xF0u ? 0x90u : 0x80u, b0 == 0xF4u ? 0x8Fu : 0xBFu) &&
             cont(b2, 0x80u, 0xBFu) && cont(b3, 0x80u, 0xBFu)) {
    cp = ((b0 & 0x07u) << 18) | ((b1 & 0x3Fu) << 12) | ((b2 & 0x3Fu) << 6) | (b3 & 0x3Fu);
    len = 4;
  } else {
    return kPrNo;
  }
  // both table walks issued together (index loads, then data loads)
  const uint32_t ci = kUcClassIndex[cp >> 8], li = kUcLowerIndex[cp >> 8];
  const uint32_t cls = kUcClassData[ci * 256u + (cp & 255u)];
  const int32_t dl = kUcLowerData[li * 256u + (cp & 255u)];
  if (cls == kUcALetter) {
    if (dl == 0) return kPrLetter | (len << 4);
    const uint32_t lc = (uint32_t)((int32_t)cp + dl);
    const uint32_t ll = lc < 0x80u ? 1u : (lc < 0x800u ? 2u : (lc < 0x10000u ? 3u : 4u));
    if (ll != len || len > 3 || uc_class(lc) != kUcALetter || uc_lower(lc) != lc) return kPrNo;
    const uint32_t by = len == 2 ? ((0xC0u | (lc >> 6)) | ((0x80u | (lc & 0x3Fu)) << 8))
                                 : ((0xE0u | (lc >> 12)) | ((0x80u | ((lc >> 6) & 0x3Fu)) << 8) |
                                    ((0x80u | (lc & 0x3Fu)) << 16));
    return kPrUpper | (len << 4) | (by << 8);
  }
  if (cls == kUcOther) return kPrSep | (len << 4);
  if (cls == kUcMidLetter) return kPrMidL | (len << 4);
  if (cls == kUcMidNum) return kPrMidN | (len << 4);
  if (cls == kUcMidNumLet) return kPrMidNL | (len << 4);
  return kPrNo;
}

// UNI: per-wave bitmaps of the common non-ASCII chars, so most of them take
// no table walk: 2-byte chars (U+0080..U+07FF; lane l holds U+0080 + 32 l ..
// + 31, lanes >= 60 none) that are ALetters and their own lower case
// (simple2) or of class Other (other2); General Punctuation U+2000..U+207F
// (curly quotes, dashes, ellipsis) two bits each in lanes 0..7 (punct):
// 1 class Other, 2 MidNumLet, 3 MidLetter, 0 through the tables.
__device__ __forceinline__ void uni_prose_bitmaps(uint32_t lane, uint32_t *simple2, uint32_t *other2, uint32_t *punct) {
  uint32_t bm = 0, om = 0;
  const uint32_t c0 = min(0x80u + 32u * lane, 0x7E0u);
  const uint32_t ci = kUcClassIndex[c0 >> 8], li = kUcLowerIndex[c0 >> 8];   // 32-aligned: one table row
#pragma unroll 8
  for (uint32_t b = 0; b < 32; b++) {
    const uint32_t cp = c0 + b;
    const uint32_t cls = kUcClassData[ci * 256u + (cp & 255u)];
    bm |= (cls == kUcALetter && kUcLowerData[li * 256u + (cp & 255u)] == 0 ? 1u : 0u) << b;
    om |= (cls == kUcOther ? 1u : 0u) << b;
  }
  *simple2 = lane >= 60 ? 0u : bm;
  *other2 = lane >= 60 ? 0u : om;
  uint32_t pm = 0;
  const uint32_t g0 = 0x2000u + 16u * (lane & 7u), gi = kUcClassIndex[g0 >> 8];
#pragma unroll 4
  for (uint32_t b = 0; b < 16; b++) {
    const uint32_t cls = kUcClassData[gi * 256u + ((g0 + b) & 255u)];
    const uint32_t code = cls == kUcOther ? 1u : (cls == kUcMidNumLet ? 2u : (cls == kUcMidLetter ? 3u : 0u));
    pm |= code << (2 * b);
  }
  *punct = lane < 8 ? pm : 0u;
}

// UNI: does the staged window (LDS bytes [0, wl), zero past wl) pass (see
// uni_prose_char)?  Lane l checks window bytes [64 l, 64 l + 64): its lead
// bytes (11xxxxxx) one per step, common chars from the wave's bitmaps, the
// others through the tables, and the wave's continuation bytes (10xxxxxx)
// must be exactly those the leads claim (no orphans).  On the way separators
// become spaces and upper-case letters their lower case in the window.  Then
// each mid char joins where UAX#29 joins it (MidLetter / MidNumLet: a letter
// on both sides, WB6/7; MidNum / MidNumLet: a digit on both sides, WB11/12)
// and is kept — its bytes >= 0x80 then read as letters, so the classifier
// makes it part of the word — or becomes spaces.  (A kept mid char never
// touches an ASCII joiner: its neighbours are letters or digits, so the
// classifier's rules around it are unchanged.)  Wave-uniform result.
__device__ __forceinline__ bool uni_window_prose(uint8_t *text, uint32_t wl, uint32_t lane, uint32_t simple2,
                                                 uint32_t other2, uint32_t punct, bool *nonascii = nullptr) {
  const uint4 *seg = reinterpret_cast<const uint4 *>(text + 64 * lane);
  uint64_t lead = 0;
  uint32_t ncont = 0;
  // the lane's four 16 B pieces in an order rotated by lane / 2: every group
  // of 8 lanes of a ds_read_b128 then covers 8 distinct bank groups (in the
  // plain order lanes 64 B apart collide: 2.2 ms of cfg-2 prose in this step)
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t qq = (q + (lane >> 1)) & 3u;
    const uint4 v = seg[qq];
    const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
    uint32_t m16 = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t x = xs[i], hb = x & 0x80808080u, ld = hb & (x << 1);
      ncont += (uint32_t)__popc(hb & ~ld);
      m16 |= swar_nib(ld) << (4 * i);
    }
    lead |= (uint64_t)m16 << (16 * qq);
  }
  if (nonascii) *nonascii = __any(lead != 0) || __any(ncont != 0);
  const uint32_t *tw = reinterpret_cast<const uint32_t *>(text);
  bool ok = true;
  uint32_t claimed = 0;
  uint64_t ml = 0, mn = 0, m3 = 0;
  while (__any(lead != 0)) {                            // one lead per lane per step
    const bool has = lead != 0;
    const uint32_t bt = has ? (uint32_t)__builtin_ctzll(lead) : 0u, pos = 64 * lane + bt;
    lead &= lead - 1;
    const uint32_t w = __builtin_amdgcn_alignbyte(tw[(pos >> 2) + 1], tw[pos >> 2], pos & 3);
    const uint32_t b0 = w & 0xFFu, b1 = (w >> 8) & 0xFFu, b2 = (w >> 16) & 0xFFu;
    const bool two = has && b0 >= 0xC2u && b0 < 0xE0u && (b1 & 0xC0u) == 0x80u && wl - pos >= 2;
    const bool gp = has && b0 == 0xE2u && (b1 == 0x80u || b1 == 0x81u) && (b2 & 0xC0u) == 0x80u && wl - pos >= 3;
    const uint32_t cp = ((b0 & 0x1Fu) << 6) | (b1 & 0x3Fu), gi = ((b1 & 1u) << 6) | (b2 & 0x3Fu);
    const int src2 = two ? (int)((cp - 0x80u) >> 5) : 0;
    const uint32_t sb = (uint32_t)__shfl((int)simple2, src2, 64), ob = (uint32_t)__shfl((int)other2, src2, 64);
    const uint32_t pb = (uint32_t)__shfl((int)punct, gp ? (int)(gi >> 4) : 0, 64);
    const uint32_t pc = (pb >> (2 * (gi & 15u))) & 3u;
    uint32_t kind = kPrNo, len = 0, lw = 0;
    if (two && ((sb >> (cp & 31u)) & 1u)) { kind = kPrLetter; len = 2; }
    else if (two && ((ob >> (cp & 31u)) & 1u)) { kind = kPrSep; len = 2; }
    else if (gp && pc) { kind = pc == 1u ? kPrSep : (pc == 2u ? kPrMidNL : kPrMidL); len = 3; }
    else if (has) {
      const uint32_t r = uni_prose_char(w, wl - pos);
      kind = r & 15u;
      len = (r >> 4) & 15u;
      lw = r >> 8;
    }
    ok &= !has || kind != kPrNo;
    if (kind == kPrSep)
      for (uint32_t i = 0; i < len; i++) text[pos + i] = 0x20u;
    else if (kind == kPrUpper)
      for (uint32_t i = 0; i < len; i++) text[pos + i] = (uint8_t)(lw >> (8 * i));
    const uint64_t bit = 1ull << bt;
    if (kind == kPrMidL || kind == kPrMidNL) ml |= bit;
    if (kind == kPrMidN || kind == kPrMidNL) mn |= bit;
    if (len == 3) m3 |= bit;
    claimed += len ? len - 1 : 0u;
  }
  if (!(__all(ok) && wave_sum(claimed) == wave_sum(ncont))) return false;
  // mid chars: the window now holds lowered letters and spaced separators; a
  // neighbour byte >= 0x80 is a letter unless it belongs to another mid char
  const uint64_t mid = ml | mn, mid3 = mid & m3;
  if (__any(mid != 0)) {
    __syncthreads();                                    // (one-wave workgroup) the rewrites above are visible
    // neighbours' mid leads across the lane edges (shuffles unconditional: a
    // lane outside EXEC reads as 0)
    const uint64_t pm = (uint64_t)__shfl_up((long long)mid, 1, 64), pm3 = (uint64_t)__shfl_up((long long)mid3, 1, 64);
    const uint64_t nm = (uint64_t)__shfl_down((long long)mid, 1, 64);
    const uint64_t P = lane ? pm : 0ull, P3 = lane ? pm3 : 0ull, N = lane < 63 ? nm : 0ull;
    uint64_t m = mid, drop = 0;
    while (m) {
      const uint32_t b = (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      const uint32_t len = ((mid3 >> b) & 1u) ? 3u : 2u, pos = 64 * lane + b;
      // mid lead bits at offsets -2 (2-byte char) / -3 (3-byte char) and +len
      const auto midat = [&](int o, bool three) -> bool {
        const int q = (int)b + o;
        const uint64_t mm = three ? (q < 0 ? P3 : mid3) : (q < 0 ? P : (q < 64 ? mid : N));
        const uint32_t qq = (uint32_t)(q < 0 ? q + 64 : (q < 64 ? q : q - 64));
        return (mm >> qq) & 1u;
      };
      const uint32_t pb = pos ? text[pos - 1] : 0u, nb = text[pos + len];
      const bool pmid = pb >= 0x80u && (midat(-2, false) || midat(-3, true));
      const bool nmid = nb >= 0x80u && midat((int)len, false);
      const bool pl = (pb >= 0x80u && !pmid) || ((pb | 0x20u) - 0x61u < 26u);
      const bool nl = (nb >= 0x80u && !nmid) || ((nb | 0x20u) - 0x61u < 26u);
      const bool pd = pb - 0x30u < 10u, nd = nb - 0x30u < 10u;
      const bool join = (((ml >> b) & 1u) && pl && nl) || (((mn >> b) & 1u) && pd && nd);
      if (!join) drop |= 1ull << b;
    }
    __syncthreads();                                    // every decision read the window as it was
    while (drop) {
      const uint32_t b = (uint32_t)__builtin_ctzll(drop);
      drop &= drop - 1;
      const uint32_t len = ((mid3 >> b) & 1u) ? 3u : 2u, pos = 64 * lane + b;
      for (uint32_t i = 0; i < len; i++) text[pos + i] = 0x20u;
    }
    __syncthreads();
  }
  return true;
}

// Units: PACK = false, one document per unit (documents 0..n_docs-1, or the
// doc_list entries); PACK = true, unit u = documents [u * pack, u * pack + pack)
// sharing one window.  A pack that cannot take the packed path (window or
// token/term capacity, non-contiguous sources, an empty or non-ASCII document)
// sends its documents to retry_list for a PACK = false pass.
#ifndef TFIDF_WAVE_XCD
#define TFIDF_WAVE_XCD 1
#endif

// UNI = true (round 5): the documents the ASCII pass flagged (uni_list), one
// wave each, by the same rules with non-ASCII bytes read as letters when
// uni_simple_span passes the document (its flag is then cleared); the rest
// stay flagged for k_tokenize_uwave.
template <bool PACK, bool G4, bool UNI = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_tokenize_wave(BuildParams p) {
  __shared__ WaveSmem sm;
  const uint32_t lane = threadIdx.x;
  clear_table(sm, lane);           // table starts empty; every document leaves it empty
  init_sel_table(sm.sel, lane);
  unsigned long long my_doc_count = 0, my_ttf = 0, my_nnz = 0;
  uint4 v[4] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  const uint64_t n_units = PACK ? (p.n_docs + p.pack - 1) / p.pack : (TFIDF_COLD(doc_list) ? *TFIDF_COLD(doc_list_count) : p.n_docs);
  // Units of this workgroup: XCD x (= workgroup mod 8, the dispatch order)
  // takes the contiguous eighth [x, x + 1) * n_units / 8 of the units, so
  // the documents running together on one XCD are neighbours and the CSR
  // lines their rows share are completed in that XCD's L2.
  const bool xm = TFIDF_WAVE_XCD && (gridDim.x & 7u) == 0 && n_units >= gridDim.x;
  const uint64_t per = (n_units + 7) / 8;
  const uint64_t ubeg = xm ? (blockIdx.x & 7u) * per + (blockIdx.x >> 3) : blockIdx.x;
  const uint64_t uend = xm ? min(n_units, ((blockIdx.x & 7u) + 1) * per) : n_units;
  const uint64_t ustep = xm ? gridDim.x >> 3 : gridDim.x;
  // UNI: units = the flagged documents, 64 flags per ballot (workgroup b
  // takes flag chunks b, b + grid, ...); kNoUnit ends.  The only state kept
  // across documents is the current chunk's remaining flags (fmk): the chunk
  // base is the current document's (SGPRs are the scarce resource here).
  constexpr uint64_t kNoUnit = ~0ull;
  uint64_t fmk = 0;
  uint32_t my_uni = 0;                                      // lane 0 counts (a VGPR)
  auto uni_scan = [&](uint64_t cb) __attribute__((always_inline)) -> uint64_t {
    for (; cb < p.n_docs; cb += (uint64_t)gridDim.x * 64) {
      fmk = __ballot(cb + lane < p.n_docs && TFIDF_COLD(uni_list)[cb + lane] != 0u);
      if (fmk) {
        const uint64_t dd = cb + (uint64_t)__builtin_ctzll(fmk);
        fmk &= fmk - 1;
        return dd;
      }
    }
    return kNoUnit;
  };
  auto uni_next = [&](uint64_t cur) __attribute__((always_inline)) -> uint64_t {
    if (fmk) {
      const uint64_t dd = (cur & ~63ull) + (uint64_t)__builtin_ctzll(fmk);
      fmk &= fmk - 1;
      return dd;
    }
    return uni_scan((cur & ~63ull) + (uint64_t)gridDim.x * 64);
  };
  const uint64_t u0 = UNI ? uni_scan((uint64_t)blockIdx.x * 64) : ubeg;
  uint32_t simple2 = 0, other2 = 0, punct = 0;
  if (UNI && u0 != kNoUnit) uni_prose_bitmaps(lane, &simple2, &other2, &punct);
  const uint64_t ulim = UNI ? kNoUnit : uend;
  DocMeta meta;
  if (u0 < ulim) {
    meta = unit_meta<PACK>(p, u0, lane);
    prefetch_wave(p, meta, lane, v);
  }
  const uint32_t R = p.n_ranges;
  uint16_t *slots = reinterpret_cast<uint16_t *>(sm.list);
  // PACK per-document scratch in the histogram queue area (free after the histogram)
  uint32_t *pk_len = reinterpret_cast<uint32_t *>(sm.qkey), *pk_nu = pk_len + kPackMax,
           *pk_start = pk_len + 2 * kPackMax;
  uint64_t *pk_row = sm.qkey + 2 * kPackMax;

  uint64_t unext = 0;                                       // UNI: the next flagged document
  for (uint64_t u = u0; u < ulim; u = UNI ? unext : u + ustep) {
    const uint64_t d = meta.d, src = meta.src, L = meta.L, s0 = meta.s0;
    const uint32_t shift = meta.shift, np = meta.np;
    const uint64_t pofs = meta.pofs;
    const bool fits = fits_wave(meta);
    const uint64_t un = UNI ? uni_next(u) : u + ustep;
    if (UNI) unext = un;
    if (!fits) {
      if (PACK) defer_pack(p, d, np, lane);
      else if (UNI) {}                                      // (flagged documents fit: the ASCII pass staged them)
      else if (lane == 0) TFIDF_COLD(long_list)[atomicAdd(TFIDF_COLD(long_count), 1u)] = (uint32_t)d;
      if (un < ulim) { meta = unit_meta<PACK>(p, un, lane); prefetch_wave(p, meta, lane, v); }
      continue;                                             // wave-uniform
    }
    // ---- stage: registers -> LDS (whole window; bytes outside the document
    // zeroed), then fetch the next document
    {
      const uint32_t hi_b = shift + (uint32_t)L;
      const uint32_t nchunks = (hi_b + 15) >> 4;
      uint4 *dst = reinterpret_cast<uint4 *>(sm.text);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t c = lane + 64 * k;
        uint4 val = c < nchunks ? v[k] : make_uint4(0, 0, 0, 0);
        if (c == 0 || c == nchunks - 1) {
          val.x &= keep_range(16 * c, shift, hi_b);
          val.y &= keep_range(16 * c + 4, shift, hi_b);
          val.z &= keep_range(16 * c + 8, shift, hi_b);
          val.w &= keep_range(16 * c + 12, shift, hi_b);
        }
        dst[c] = val;
        v[k] = val;                                         // classified from registers below
      }
    }
    asm volatile("" ::: "memory");

    // ---- classify (window chunks in registers) + spans -> dense token list
    bool bad, under;
    uint64_t wbase = 0;
    bool upper;
    uint64_t W;
    if constexpr (UNI) {
      // flagged document: the prose check rewrites the staged window, whose
      // chunks are read back into the registers (lane l: chunks l + 64 k, no
      // bank conflicts) and classified there as an ASCII window is; then the
      // next window's fetch goes out
      // (round 6 first form: classified from LDS by 64-byte lane segments,
      // with the mid chars joined in the classifier — 2.3 ms of cfg-2 prose
      // in that step alone, the strided 16 B reads' bank conflicts)
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = make_uint4(0, 0, 0, 0);   // (staged: no registers held over the check)
      bool na;                                              // (UNI-first builds: ASCII documents come here too)
      const bool pass = uni_window_prose(sm.text, shift + (uint32_t)L, lane, simple2, other2, punct, &na);
      if (!pass || p.debug_stop == 5) {                     // (profiling stops 5, 6: this pass's phases)
        if (un < ulim) { meta = unit_meta<PACK>(p, un, lane); prefetch_wave(p, meta, lane, v); }
        if (pass && lane == 0) TFIDF_COLD(uni_list)[d] = 0u;
        continue;
      }
      if (lane == 0) TFIDF_COLD(uni_list)[d] = 0u;           // taken here (else: k_tokenize_uwave)
      my_uni += lane == 0 && na;
      __syncthreads();                                      // (one wave) the window's rewrites are visible
      {
        const uint4 *src = reinterpret_cast<const uint4 *>(sm.text);
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = src[lane + 64 * k];
      }
      const uint32_t nrows = (shift + (uint32_t)L + 1023) >> 10;
      uint16_t *wm16 = reinterpret_cast<uint16_t *>(sm.qkey);            // (histogram queue: written before read)
      W = regs_word_mask<false, true>(v, nrows, sm.text, wm16, wm16 + 256, lane, &bad, &under, &wbase, &upper);
      bad = false;
      if (un < ulim) { meta = unit_meta<PACK>(p, un, lane); prefetch_wave(p, meta, lane, v); }
      if (p.debug_stop == 6) continue;
    } else {
      // a byte >= 0x80 (in the staged registers): the document goes to the UNI
      // pass unclassified (nrows 0; flagged below as `bad`)
      bool skipc = false;
      if (!UNI && !PACK) {
        uint32_t hx = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) hx |= v[k].x | v[k].y | v[k].z | v[k].w;
        skipc = __any((hx & 0x80808080u) != 0);
      }
      const uint32_t nrows = skipc ? 0u : (shift + (uint32_t)L + 1023) >> 10;
      uint16_t *wm16 = reinterpret_cast<uint16_t *>(sm.list);            // the token list is written after
      W = regs_word_mask<PACK>(v, nrows, sm.text, wm16, wm16 + 256, lane, &bad, &under, &wbase, &upper);
      bad |= skipc;
      // the next document's window, now that this one's registers are consumed
      if (un < ulim) { meta = unit_meta<PACK>(p, un, lane); prefetch_wave(p, meta, lane, v); }
    }
    asm volatile("" ::: "memory");
    if (p.debug_stop == 1) continue;
    // PACK: document boundaries q_j (window position of document j's first
    // byte, j >= 1).  No token spans one: a joiner next to q_j that is a word
    // byte only through its neighbour across q_j is dropped, and a token is
    // ended / started at q_j.  Token -> document: dbase = #{q_j <= 64 lane} plus
    // the boundaries inside the lane below the token start (bm).
    uint64_t bq = 0, bm = 0;
    uint32_t dbase = 0;
    if (PACK && !bad) {
      const uint32_t qv = shift + (uint32_t)(pofs - s0);
      uint64_t jm = 0;
      const uint32_t l0 = 64 * lane;
      for (uint32_t j = 1; j < np; j++) {
        const uint32_t q = (uint32_t)__builtin_amdgcn_readlane((int)qv, (int)j);
        dbase += q <= l0;
        const uint32_t r = q - l0;                           // wraps for q < l0
        if (r < 64) { bq |= 1ull << r; if (r) bm |= 1ull << r; }
        if (r - 1 < 64) jm |= 1ull << (r - 1);
        if (r < 64) jm |= 1ull << r;
      }
      W &= ~(jm & ~wbase);
    }
    if (bad) {                                              // non-ASCII: the Unicode wave path
      if (PACK) defer_pack(p, d, np, lane);
      else if (lane == 0) flag_unicode(TFIDF_COLD(uni_list), d);
      continue;
    }
    const uint64_t wlast = __ballot((W >> 63) & 1ull);
    const uint64_t prevW = lane ? (wlast >> (lane - 1)) & 1ull : 0ull;
    uint64_t S = W & ~((W << 1) | prevW);
    uint64_t E = ~W & ((W << 1) | prevW);
    if (PACK) {
      S |= bq & W;
      E |= bq & ((W << 1) | prevW);
    }
    const uint32_t firstE = E ? lane * 64 + (uint32_t)__builtin_ctzll(E) : kWaveWindow;
    const uint64_t hasE = __ballot(E != 0);
    const uint64_t later = lane == 63 ? 0ull : (hasE & (~0ull << (lane + 1)));
    const uint32_t srcl = later ? (uint32_t)__builtin_ctzll(later) : lane;
    uint32_t nz = (uint32_t)__shfl((int)firstE, (int)srcl, 64);
    if (!later) nz = kWaveWindow;
    if (prevW) E &= E - 1;                                  // closes the token open from lane - 1
    const uint32_t nts = (uint32_t)__popcll(S);
    const uint32_t tincl = wave_incl_add(nts);
    const uint32_t ntok = (uint32_t)__builtin_amdgcn_readlane((int)tincl, 63);
    if (ntok > kWaveTokens) {                               // wave-uniform
      if (PACK) defer_pack(p, d, np, lane);
      else if (lane == 0) TFIDF_COLD(long_list)[atomicAdd(TFIDF_COLD(long_count), 1u)] = (uint32_t)d;
      continue;
    }
    bool longtok = false;
    {
      // the k-th start pairs with the k-th end; starts of the low half first
      // (their ends in the low half, else the high half, else nz), then the
      // high half's (every low-half end is taken by then)
      uint32_t at = tincl - nts;
      uint32_t s0 = (uint32_t)S, s1 = (uint32_t)(S >> 32), e0 = (uint32_t)E, e1 = (uint32_t)(E >> 32);
      const uint32_t l64 = lane * 64;
      while (s0) {
        const uint32_t tp = l64 + (uint32_t)__builtin_ctz(s0);
        const uint32_t te = e0 ? l64 + (uint32_t)__builtin_ctz(e0) : (e1 ? l64 + 32 + (uint32_t)__builtin_ctz(e1) : nz);
        s0 &= s0 - 1;
        if (e0) e0 &= e0 - 1; else e1 &= e1 - 1;
        longtok |= te - tp > (UNI ? 7u : 8u);
        const uint32_t j = PACK ? dbase + (uint32_t)__popcll(bm & ((2ull << (tp - l64)) - 1)) : 0u;
        sm.list[at++] = span_entry(tp, te, j);
      }
      while (s1) {
        const uint32_t tp = l64 + 32 + (uint32_t)__builtin_ctz(s1);
        const uint32_t te = e1 ? l64 + 32 + (uint32_t)__builtin_ctz(e1) : nz;
        s1 &= s1 - 1;
        e1 &= e1 - 1;
        longtok |= te - tp > (UNI ? 7u : 8u);
        const uint32_t j = PACK ? dbase + (uint32_t)__popcll(bm & ((2ull << (tp - l64)) - 1)) : 0u;
        sm.list[at++] = span_entry(tp, te, j);
      }
    }
    asm volatile("" ::: "memory");
    if (p.debug_stop == 2) continue;

    // ---- per-document histogram in LDS (folded-key and '_'-only checks only
    // when the document holds a token of more than 8 bytes or a '_')
    const bool anylong = __any(longtok) || under;
    uint32_t nu = 0, len = 0;
    bool overflow = false;
    for (uint32_t tb = 0; tb < ntok && !overflow;) {       // batch width by what is left
      const uint32_t rem = ntok - tb;
      if (anylong) {
        if (TFIDF_HIST10 && !PACK && !UNI && rem > 512 && rem <= 640) { hist2<10, true, PACK, UNI>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 640; }
        else if (rem > 256) { hist2<8, true, PACK, UNI>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 512; }
        else if (rem > 128) { hist2<4, true, PACK, UNI>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 256; }
        else { hist2<2, true, PACK, UNI>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 128; }
      } else {
        // 513..640 tokens (U[400, 600]-token documents: ~40 % of cfg 2) in one batch
        if (TFIDF_HIST10 && !PACK && !UNI && rem > 512 && rem <= 640) { hist2<10, false, PACK>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 640; }
        else if (rem > 256) { hist2<8, false, PACK>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 512; }
        else if (rem > 128) { hist2<4, false, PACK>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 256; }
        else { hist2<2, false, PACK>(sm, lane, tb, ntok, under, upper, nu, len, overflow); tb += 128; }
      }
    }
    if (overflow || nu > kWaveTerms) {                      // wave-uniform: long path
      clear_table(sm, lane);
      if (PACK) defer_pack(p, d, np, lane);
      else if (lane == 0) TFIDF_COLD(long_list)[atomicAdd(TFIDF_COLD(long_count), 1u)] = (uint32_t)d;
      continue;
    }
    if (p.debug_stop == 3) { clear_table(sm, lane); continue; }

    // ---- dense list of occupied table slots (this lane scans 16)
    {
      uint32_t occ = 0;
      const uint4 *kp = reinterpret_cast<const uint4 *>(&sm.key[16 * lane]);
      // lanes are 128 B apart: visiting the 16-B pieces in an order rotated by
      // (lane >> 1) & 7 gives every ds_read_b128 lane group 16 distinct bank
      // slots (unrotated: 8-way conflicts, most of the kernel's conflict cycles)
      const uint32_t rot = (lane >> 1) & 7;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const uint32_t qq = (q + rot) & 7;
        const uint4 t = kp[qq];
        occ |= ((uint32_t)((t.x | t.y) != 0) | ((uint32_t)((t.z | t.w) != 0) << 1)) << (2 * qq);
      }
      const uint32_t c = (uint32_t)__popc(occ);
      uint32_t at = wave_incl_add(c) - c;
      while (occ) {
        slots[at++] = (uint16_t)(16 * lane + (uint32_t)__builtin_ctz(occ));
        occ &= occ - 1;
      }
      asm volatile("" ::: "memory");
    }

    // ---- dictionary slots of terms lane + 64k
    uint32_t g[kWaveK], tf[kWaveK], tdoc[kWaveK];
    uint32_t actm = 0;
    resolve_terms<PACK, G4, UNI>(sm, p, lane, nu, (uint32_t)d, g, tf, tdoc, actm, pk_len, pk_nu, s0 - shift,
                                 shift + (uint32_t)L);
    if (p.debug_stop == 4) { clear_table(sm, lane); continue; }

    // ---- CSR row grouped by dictionary range (PACK: by (document, range)),
    // staged in LDS.  G <= kWaveGroups groups (host: pack <= kWaveGroups / R).
    uint32_t *st_col = reinterpret_cast<uint32_t *>(sm.key);
    uint32_t *st_tf = st_col + kWaveSlots;
    const uint32_t st_noop = kWaveSlots - 64 + lane;          // unused staging words (nu <= kWaveTerms)
    // PACK: groups are (document, range) in that order, so each document's row
    // is one contiguous run of the staging area starting at pk_start[j]
    const uint32_t rbits = (uint32_t)__builtin_ctz(R);
    const uint32_t G = PACK ? np << rbits : R;
    if (PACK && G > kWaveGroups) {                          // cannot happen (host pack limit)
      clear_table(sm, lane);
      defer_pack(p, d, np, lane);
      continue;
    }
    if (PACK) {
      const uint32_t nuj = lane < np ? pk_nu[lane] : 0u;
      const uint32_t incl = wave_incl_add(nuj);
      if (lane < np) {
        pk_start[lane] = incl - nuj;
        pk_row[lane] = (pofs + src + lane) >> 1;             // csr_row_base of document src + lane
      }
    }
    // Group ranks by LDS atomics on per-group counters in the count array
    // (consumed by resolve_terms): [0, 128) counters, then exclusive group
    // bases; idle terms bump no-op counters [128, 192).  Order inside a
    // (document, range) segment is free (one entry per slot).  Replaces the
    // packed 16-bit range-field wave scans of round 2 (~20 -> ~8 VALU per term).
    static_assert(kWaveGroups == 128 && kWaveSlots / 2 >= 192, "group counters");
    uint32_t *gcnt = sm.cnt;
    gcnt[lane] = 0;
    gcnt[lane + 64] = 0;
    uint32_t grp[kWaveK], rank[kWaveK];
#pragma unroll
    for (int k = 0; k < (int)kWaveK; k++) {
      const bool act = (actm >> k) & 1u;
      grp[k] = act ? (PACK ? (tdoc[k] << rbits) + (g[k] >> p.range_shift) : (g[k] >> p.range_shift)) : 128u + lane;
      rank[k] = atomicAdd(&gcnt[grp[k]], 1u);
    }
    const uint32_t c0 = gcnt[lane], c1 = gcnt[lane + 64];
    const uint32_t i0 = wave_incl_add(c0);
    const uint32_t i1 = wave_incl_add(c1) + (uint32_t)__builtin_amdgcn_readlane((int)i0, 63);
    gcnt[lane] = i0 - c0;
    gcnt[lane + 64] = i1 - c1;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t gg = lane + 64 * h, e = h ? i1 : i0;
      if (gg < G) {
        if (PACK) p.rsplit[(d + (gg >> rbits)) * R + (gg & (R - 1))] = e - pk_start[gg >> rbits];
        else p.rsplit[d * R + gg] = e;
      }
    }
#pragma unroll
    for (int k = 0; k < (int)kWaveK; k++) {
      const bool act = (actm >> k) & 1u;
      const uint32_t pos = act ? gcnt[grp[k]] + rank[k] : st_noop;
      st_col[pos] = g[k];
      st_tf[pos] = PACK ? tf[k] | (tdoc[k] << 24) : tf[k];
    }
    asm volatile("" ::: "memory");
    if (PACK) {
      for (uint32_t i = lane; i < nu; i += 64) {
        const uint32_t t = st_tf[i], j = t >> 24;
        csr_put(p, pk_row[j] + i - pk_start[j], st_col[i], t & 0xFFFFFFu, (uint32_t)(d + j));
      }
      if (lane < np) {
        const uint32_t lj = pk_len[lane], nj = pk_nu[lane];
        p.doc_len[d + lane] = lj;
        p.doc_nuniq[d + lane] = nj;
        p.doc_norm[d + lane] = (uint8_t)int_to_byte4(lj);
        my_doc_count += lj > 0;
        my_ttf += lj;
        my_nnz += nj;
      }
      clear_table(sm, lane);
      continue;
    }
    {
      const uint64_t row = csr_row_base(p.offsets, src);
      for (uint32_t i = lane; i < nu; i += 64) csr_put(p, row + i, st_col[i], st_tf[i], (uint32_t)d);
    }
    clear_table(sm, lane);
    if (lane == 0) {
      p.doc_len[d] = len;
      p.doc_nuniq[d] = nu;
      p.doc_norm[d] = (uint8_t)int_to_byte4(len);
      my_doc_count += len > 0;
      my_ttf += len;
      my_nnz += nu;
    }
  }
  if (my_ttf | my_nnz | my_doc_count) {                    // lane 0 (PACK: lanes < pack)
    atomicAdd(&TFIDF_COLD(stats)[0], my_doc_count);
    atomicAdd(&TFIDF_COLD(stats)[1], my_ttf);
    atomicAdd(&TFIDF_COLD(stats)[2], my_nnz);
  }
  if (UNI && my_uni) atomicAdd(TFIDF_COLD(uni_wave_count), my_uni);   // lane 0
}

// ---------------------------------------------------------------------------
// Book-sized documents (SURVEY cfg 1), ASCII: chunk-parallel.  A long
// document is cut into kCoreBytes cores; unit = (document, core).  A wave
// stages the core with kPreBytes of context before it and kPostBytes after it
// (UAX#29 decisions look at most two characters around a position; a token
// that runs past the post margin is longer than 255 characters), keeps the
// tokens STARTING in its core, counts them in its LDS table, resolves the
// distinct terms in the global dictionary (resolve_terms) and stores them as
// the unit's pair list ((slot within bucket) << kPairTfBits | tf), grouped by
// slot bucket (slot >> pair_bshift; bucket starts in pair_ub).  k_long_rows
// then sums each document's pair lists window by window in LDS into its CSR
// row.  (Round 2 added the counts into a dense per-document array in HBM with
// global atomics: ~20 M scattered memory-side atomics per 300-book build cost
// 0.43 of the 1.29 ms, and scanning the 1 MB arrays another 0.26.)  A chunk
// that cannot take this path (non-ASCII
// text, a token of more than 255 characters, more than 512 distinct terms)
// marks its document, which then goes to k_tokenize_long as a whole.
// UNI = true (round 5): the units this kernel flagged for non-ASCII text
// (uchunk_list), by the same rules with non-ASCII bytes read as letters when
// uni_window_simple passes the window (its flag is then cleared); the rest
// stay flagged for k_tokenize_uchunk.
template <bool UNI = false>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_tokenize_chunk(BuildParams p) {
  __shared__ WaveSmem sm;
  const uint32_t lane = threadIdx.x;
  clear_table(sm, lane);
  init_sel_table(sm.sel, lane);
  uint4 v[4] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
  const uint64_t n_units = p.n_chunks;
  uint16_t *slots = reinterpret_cast<uint16_t *>(sm.list);
  ChunkMeta meta;
  auto prefetch = [&](const ChunkMeta &m) {
    const uint32_t nchunks = (uint32_t)((m.shift + m.L + 15) >> 4);
    const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(p.text + m.s0) & ~(uintptr_t)15);
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (lane + 64 * k < nchunks) v[k] = gload16(src + lane + 64 * k);
  };
  uint32_t my_uc = 0;                                        // units this wave flagged for k_tokenize_uchunk
  // UNI: the flagged units of this workgroup's stride
  auto next_flagged = [&](uint64_t v) __attribute__((always_inline)) -> uint64_t {
    while (v < n_units && p.uchunk_list[v] == 0) v += gridDim.x;
    return v;
  };
  if (UNI && *p.uchunk_count == 0) return;                   // wave-uniform
  const uint64_t u0 = UNI ? next_flagged(blockIdx.x) : blockIdx.x;
  uint32_t simple2 = 0, other2 = 0, punct = 0;
  if (UNI && u0 < n_units) uni_prose_bitmaps(lane, &simple2, &other2, &punct);
  if (u0 < n_units) { meta = chunk_meta(p, u0); prefetch(meta); }
  uint64_t un = 0;
  for (uint64_t u = u0; u < n_units; u = un) {
    const ChunkMeta m = meta;
    un = UNI ? next_flagged(u + gridDim.x) : u + gridDim.x;
    uint32_t hib = 0;                                          // OR of the window's bytes: bit 7s = non-ASCII
    {   // stage (bytes outside the window zeroed), then fetch the next unit
      const uint32_t hi_b = m.shift + (uint32_t)m.L;
      const uint32_t nchunks = (hi_b + 15) >> 4;
      uint4 *dst = reinterpret_cast<uint4 *>(sm.text);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t c = lane + 64 * k;
        uint4 val = c < nchunks ? v[k] : make_uint4(0, 0, 0, 0);
        if (c == 0 || c == nchunks - 1) {
          val.x &= keep_range(16 * c, m.shift, hi_b);
          val.y &= keep_range(16 * c + 4, m.shift, hi_b);
          val.z &= keep_range(16 * c + 8, m.shift, hi_b);
          val.w &= keep_range(16 * c + 12, m.shift, hi_b);
        }
        hib |= val.x | val.y | val.z | val.w;
        dst[c] = val;
      }
    }
    if (un < n_units) { meta = chunk_meta(p, un); prefetch(meta); }
    asm volatile("" ::: "memory");
    const uint32_t fail_at = m.gi;
    // non-ASCII text (the classifier's own test, from the staged registers, so
    // such a unit is not classified here): flagged for the Unicode chunk kernel
    // (a flag per unit, counted once per wave at the end — a list appended
    // with one atomic per unit serialised 15 k units on one counter)
    const bool nonascii = __any((hib & 0x80808080u) != 0);
    if (UNI && nonascii) {                                     // simple non-ASCII text: taken here
      // A window that starts or ends inside its document can cut a multi-byte
      // char in its margin: those bytes are blanked (class Other) — they lie
      // 64 bytes before the core or 320 after it, so the core's tokens keep
      // their boundaries (round 6: prose books sent such units to
      // k_tokenize_uchunk, ~0.36 ms)
      if (lane == 0) {
        const uint64_t src = p.live_map ? p.live_map[m.d] : m.d;
        uint8_t *t = sm.text + m.shift;
        const uint32_t L = (uint32_t)m.L;
        if (m.s0 > p.offsets[src])
          for (uint32_t i = 0; i < 3 && i < L && (t[i] & 0xC0u) == 0x80u; i++) t[i] = 0;
        if (m.s0 + m.L < p.offsets[src + 1])
          for (uint32_t j = 1; j <= 3 && j <= L; j++) {
            const uint32_t c = t[L - j];
            if ((c & 0xC0u) == 0xC0u) {                        // the last lead: is its char complete?
              const uint32_t need = c >= 0xF0u ? 4u : (c >= 0xE0u ? 3u : 2u);
              if (need > j)
                for (uint32_t i = L - j; i < L; i++) t[i] = 0;
              break;
            }
            if ((c & 0x80u) == 0) break;
          }
      }
      __syncthreads();
      if (!uni_window_prose(sm.text, m.shift + (uint32_t)m.L, lane, simple2, other2, punct))
        continue;                                              // k_tokenize_uchunk
      if (lane == 0) p.uchunk_list[u] = 0u;
    } else if (nonascii) {
      if (lane == 0) {
        if (p.uchunk_list) { p.uchunk_list[u] = 1u; my_uc++; }
        else p.chunk_fail[fail_at] = 1u;
      }
      continue;
    }
    bool bad, under;
    uint64_t wbase = 0;
    bool upper;
    const uint64_t W = lane_word_mask<false, UNI>(sm.text, lane, &bad, &under, &wbase, &upper);
    const uint64_t wlast = __ballot((W >> 63) & 1ull);
    const uint64_t prevW = lane ? (wlast >> (lane - 1)) & 1ull : 0ull;
    const uint64_t S = W & ~((W << 1) | prevW);
    uint64_t E = ~W & ((W << 1) | prevW);
    const uint32_t firstE = E ? lane * 64 + (uint32_t)__builtin_ctzll(E) : kWaveWindow;
    const uint64_t hasE = __ballot(E != 0);
    const uint64_t later = lane == 63 ? 0ull : (hasE & (~0ull << (lane + 1)));
    const uint32_t srcl = later ? (uint32_t)__builtin_ctzll(later) : lane;
    uint32_t nz = (uint32_t)__shfl((int)firstE, (int)srcl, 64);
    if (!later) nz = kWaveWindow;
    if (prevW) E &= E - 1;
    // tokens starting in the core only: buffer positions [A, B)
    const uint32_t A = m.shift + m.core_lo, B = m.shift + m.core_hi, l0 = 64 * lane;
    const uint64_t below_b = B <= l0 ? 0ull : (B - l0 >= 64 ? ~0ull : ((1ull << (B - l0)) - 1));
    const uint64_t below_a = A <= l0 ? 0ull : (A - l0 >= 64 ? ~0ull : ((1ull << (A - l0)) - 1));
    const uint64_t core = below_b & ~below_a;
    const uint32_t nts = (uint32_t)__popcll(S & core);
    const uint32_t tincl = wave_incl_add(nts);
    const uint32_t ntok = (uint32_t)__builtin_amdgcn_readlane((int)tincl, 63);
    bool longtok = false;
    {
      uint32_t at = tincl - nts;
      uint32_t s0 = (uint32_t)S, s1 = (uint32_t)(S >> 32), e0 = (uint32_t)E, e1 = (uint32_t)(E >> 32);
      while (s0 | s1) {
        const uint32_t tp = lane * 64 + (s0 ? (uint32_t)__builtin_ctz(s0) : 32 + (uint32_t)__builtin_ctz(s1));
        const uint32_t te = (e0 | e1) ? lane * 64 + (e0 ? (uint32_t)__builtin_ctz(e0) : 32 + (uint32_t)__builtin_ctz(e1))
                                      : nz;
        if (s0) s0 &= s0 - 1; else s1 &= s1 - 1;
        if (e0) e0 &= e0 - 1; else e1 &= e1 - 1;
        if (tp >= A && tp < B) {
          longtok |= te - tp > (UNI ? 7u : 8u);
          sm.list[at++] = span_entry(tp, te, 0);
        }
      }
    }
    asm volatile("" ::: "memory");
    const bool anylong = __any(longtok) || under;
    uint32_t nu = 0, toks = 0;
    bool overflow = false;
    for (uint32_t tb = 0; tb < ntok && !overflow;) {
      const uint32_t rem = ntok - tb;
      if (anylong) {
        if (rem > 256) { hist2<8, true, false, UNI>(sm, lane, tb, ntok, under, upper, nu, toks, overflow); tb += 512; }
        else if (rem > 128) { hist2<4, true, false, UNI>(sm, lane, tb, ntok, under, upper, nu, toks, overflow); tb += 256; }
        else { hist2<2, true, false, UNI>(sm, lane, tb, ntok, under, upper, nu, toks, overflow); tb += 128; }
      } else {
        if (rem > 256) { hist2<8, false, false>(sm, lane, tb, ntok, under, upper, nu, toks, overflow); tb += 512; }
        else if (rem > 128) { hist2<4, false, false>(sm, lane, tb, ntok, under, upper, nu, toks, overflow); tb += 256; }
        else { hist2<2, false, false>(sm, lane, tb, ntok, under, upper, nu, toks, overflow); tb += 128; }
      }
    }
    if (overflow || nu > kWaveTerms) {
      clear_table(sm, lane);
      if (lane == 0) p.chunk_fail[fail_at] = 1u;
      continue;
    }
    {   // dense list of occupied table slots
      uint32_t occ = 0;
      const uint4 *kp = reinterpret_cast<const uint4 *>(&sm.key[16 * lane]);
      const uint32_t rot = (lane >> 1) & 7;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const uint32_t qq = (q + rot) & 7;
        const uint4 t = kp[qq];
        occ |= ((uint32_t)((t.x | t.y) != 0) | ((uint32_t)((t.z | t.w) != 0) << 1)) << (2 * qq);
      }
      const uint32_t c = (uint32_t)__popc(occ);
      uint32_t at = wave_incl_add(c) - c;
      while (occ) {
        slots[at++] = (uint16_t)(16 * lane + (uint32_t)__builtin_ctz(occ));
        occ &= occ - 1;
      }
      asm volatile("" ::: "memory");
    }
    uint32_t g[kWaveK], tf[kWaveK], tdoc[kWaveK];
    uint32_t actm = 0;
    resolve_terms<false, false, UNI>(sm, p, lane, nu, (uint32_t)m.d, g, tf, tdoc, actm, nullptr, nullptr, m.s0 - m.shift,
                                     m.shift + (uint32_t)m.L);
    {   // the unit's (slot, tf) pairs, counting-sorted by slot bucket in LDS (text and retry
        // queue are dead here), stored as one contiguous run; bucket starts to pair_ub
      uint32_t *bcnt = reinterpret_cast<uint32_t *>(sm.qkey);          // [0, 64) counts, [64, 128) starts
      uint32_t *stage = reinterpret_cast<uint32_t *>(sm.text);
      const uint32_t bsh = p.pair_bshift, nb = p.pair_nb, bmask = (1u << bsh) - 1u;
      bcnt[lane] = 0;
      asm volatile("" ::: "memory");
      uint32_t rank[kWaveK];
#pragma unroll
      for (int k = 0; k < (int)kWaveK; k++) rank[k] = ((actm >> k) & 1u) ? atomicAdd(&bcnt[g[k] >> bsh], 1u) : 0u;
      asm volatile("" ::: "memory");
      const uint32_t n = bcnt[lane];
      const uint32_t incl = wave_incl_add(n);
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      bcnt[64 + lane] = incl - n;
      uint32_t *ub = p.pair_ub + u * (nb + 1);
      if (lane < nb) ub[lane] = incl - n;
      if (lane == 0) ub[nb] = total;
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < (int)kWaveK; k++)
        if ((actm >> k) & 1u) stage[bcnt[64 + (g[k] >> bsh)] + rank[k]] = ((g[k] & bmask) << kPairTfBits) | tf[k];
      asm volatile("" ::: "memory");
      uint32_t *pr = p.pairs + u * kPairWords;
      for (uint32_t i = lane; i < total; i += 64) pr[i] = stage[i];
    }
    clear_table(sm, lane);
  }
  if (my_uc) atomicAdd(p.uchunk_count, my_uc);              // lane 0
}

// One workgroup per long document of the group: its units' pair lists ->
// CSR row, window by window (kRangeSlots slots; a window never straddles a
// range, so the row stays grouped by range; order inside a window is free),
// range splits, length, norm, statistics.  Per window: LDS counters zeroed,
// the units' pairs of the window's bucket are added (below), then
// each thread takes 32 counters (8 conflict-free 16 B reads) and a
// workgroup scan places the non-zero ones.  A document some chunk could not
// take goes to long_list (k_tokenize_long).
constexpr uint32_t kLrUpt = TFIDF_LR_UPT;                   // units per thread in a segment round
constexpr uint32_t kLrUnits = kLrUpt * kLrThreads;
constexpr uint32_t kLrPer = kLrWin / kLrThreads;            // window counters per thread (emission)
__global__ void __launch_bounds__(kLrThreads) TFIDF_LR_ATTR k_long_rows(BuildParams p) {
  extern __shared__ uint32_t acc[];                       // [W] counters of the current window
  __shared__ uint32_t wsum[kLrThreads / 64];
  __shared__ uint32_t ulo[kLrUnits], upre[kLrUnits];
  __shared__ unsigned long long lsum;
  const uint32_t gi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint64_t d = p.chunk_docs[gi];
  if (p.chunk_fail[gi] != 0) {
    if (tid == 0) p.long_list[atomicAdd(p.long_count, 1u)] = (uint32_t)d;
    return;
  }
  const uint32_t C = p.cap_mask + 1;
  const uint32_t W = C < kLrWin ? C : kLrWin;             // power of two
  const uint32_t wlog = 31 - __builtin_clz(W);
  const uint32_t bsh = p.pair_bshift, nb = p.pair_nb;
  const uint64_t src = p.live_map ? p.live_map[d] : d;
  const uint64_t row = csr_row_base(p.offsets, src);
  const uint32_t RS = 1u << p.range_shift;
  const uint32_t u0 = p.chunk_pre[gi], u1 = p.chunk_pre[gi + 1];
  if (tid == 0) lsum = 0;
  for (uint32_t i = tid; i < W / 4; i += kLrThreads) reinterpret_cast<uint4 *>(acc)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  uint32_t carry = 0;
  unsigned long long my_len = 0;
  for (uint32_t t0 = 0; t0 < C; t0 += W) {
    const uint32_t j = t0 >> bsh;                                 // the window's bucket
    const uint32_t wsel = (t0 & ((1u << bsh) - 1u)) >> wlog;      // the window inside its bucket
    // the window's bucket segments of up to kLrUnits units at a time: segment
    // starts and an exclusive scan of their lengths in LDS, then the flattened
    // entries, consecutive threads on consecutive words of a segment (coalesced;
    // a thread per unit reading its own segment touched 64 lines per load), the
    // unit of each entry by binary search of the scan
    for (uint32_t ur = u0; ur < u1; ur += kLrUnits) {
      const uint32_t nr = u1 - ur < kLrUnits ? u1 - ur : kLrUnits;
      uint32_t cu[kLrUpt];
      uint32_t tsum = 0;
#pragma unroll
      for (int h = 0; h < (int)kLrUpt; h++) {
        const uint32_t i = kLrUpt * tid + h;
        cu[h] = 0;
        if (i < nr) {
          const uint32_t *ubr = p.pair_ub + (uint64_t)(ur + i) * (nb + 1);
          const uint32_t lo = ubr[j];
          cu[h] = ubr[j + 1] - lo;
          ulo[i] = lo;
        }
        tsum += cu[h];
      }
      const uint32_t tin = wave_incl_add(tsum);
      if (lane == 63) wsum[wid] = tin;
      __syncthreads();
      uint32_t tb = 0, T = 0;
      for (uint32_t w = 0; w < kLrThreads / 64; w++) {
        const uint32_t sw = wsum[w];
        if (w < wid) tb += sw;
        T += sw;
      }
      tb += tin - tsum;
#pragma unroll
      for (int h = 0; h < (int)kLrUpt; h++) {
        if (kLrUpt * tid + h < nr) upre[kLrUpt * tid + h] = tb;
        tb += cu[h];
      }
      __syncthreads();
      constexpr int kIn = TFIDF_LR_IN;
      for (uint32_t f0 = 0; f0 < T; f0 += kIn * kLrThreads) {
        uint32_t ws[kIn], at[kIn];
#pragma unroll
        for (int q = 0; q < kIn; q++) at[q] = 0;
        // last i with upre[i] <= f: the kIn searches step together (fixed trip count, their
        // LDS reads overlap; a data-dependent loop per entry ran them one after another)
        for (int step = 31 - __builtin_clz(nr); step >= 0; step--) {
#pragma unroll
          for (int q = 0; q < kIn; q++) {
            const uint32_t f = f0 + (uint32_t)q * kLrThreads + tid, m = at[q] + (1u << step);
            if (m < nr && upre[m] <= f) at[q] = m;
          }
        }
#pragma unroll
        for (int q = 0; q < kIn; q++) {
          const uint32_t f = f0 + (uint32_t)q * kLrThreads + tid;
          ws[q] = f < T ? p.pairs[(uint64_t)(ur + at[q]) * kPairWords + ulo[at[q]] + (f - upre[at[q]])] : 0u;
        }
#pragma unroll
        for (int q = 0; q < kIn; q++) {
          const uint32_t loc = ws[q] >> kPairTfBits;
          if (ws[q] && (loc >> wlog) == wsel) atomicAdd(&acc[loc & (W - 1)], ws[q] & ((1u << kPairTfBits) - 1u));
        }
      }
      __syncthreads();                                            // wsum, ulo, upre reused
    }
    __syncthreads();
    // kLrPer (<= 32) counters per thread: i = (q * kLrThreads + tid) * 4 + c
    uint32_t v[kLrPer];
    uint32_t nz = 0;
    const uint32_t nq = W / (4 * kLrThreads);                    // 16 B reads per thread (else one, partial)
#pragma unroll
    for (int q = 0; q < (int)kLrPer / 4; q++) {
      uint4 x = make_uint4(0, 0, 0, 0);
      const uint32_t i4 = (uint32_t)q * kLrThreads + tid;
      if ((uint32_t)q < nq || (q == 0 && i4 < W / 4)) {
        x = reinterpret_cast<uint4 *>(acc)[i4];
        reinterpret_cast<uint4 *>(acc)[i4] = make_uint4(0, 0, 0, 0);   // zero for the next window
      }
      v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      nz += (x.x != 0) + (x.y != 0) + (x.z != 0) + (x.w != 0);
      my_len += (unsigned long long)x.x + x.y + x.z + x.w;
    }
    const uint32_t incl = wave_incl_add(nz);
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    uint32_t base = carry, all = 0;
    for (uint32_t w = 0; w < kLrThreads / 64; w++) {
      const uint32_t sw = wsum[w];
      if (w < wid) base += sw;
      all += sw;
    }
    uint32_t at = base + incl - nz;
#pragma unroll
    for (int q = 0; q < (int)kLrPer / 4; q++)
#pragma unroll
      for (int c = 0; c < 4; c++)
        if (v[4 * q + c]) { csr_put(p, row + at, t0 + ((uint32_t)q * kLrThreads + tid) * 4 + c, v[4 * q + c], (uint32_t)d); at++; }
    carry += all;
    const uint32_t t1 = t0 + W;
    // a range ends at the window's end: its split = entries below it
    if (tid == 0 && ((t1 & (RS - 1)) == 0 || t1 == C)) p.rsplit[d * p.n_ranges + ((t1 - 1) >> p.range_shift)] = carry;
    __syncthreads();                                              // wsum and acc reused by the next window
  }
  if (my_len) atomicAdd(&lsum, my_len);
  __syncthreads();
  if (tid == 0) {
    const uint64_t len = lsum;
    const uint32_t nu = carry;
    if (len > 0xFFFFFFFFull) set_err(p.err, kErrTfTooLarge, (uint32_t)d);
    p.doc_len[d] = (uint32_t)len;
    p.doc_nuniq[d] = nu;
    p.doc_norm[d] = (uint8_t)int_to_byte4((uint32_t)len);
    atomicAdd(&p.stats[0], (unsigned long long)(len > 0));
    atomicAdd(&p.stats[1], len);
    atomicAdd(&p.stats[2], (unsigned long long)nu);
  }
}

// ---------------------------------------------------------------------------
// Long-document path: one workgroup per document, kChunk-byte chunks staged
// with context margins, per-document table in global scratch.

struct LongSmem {
  uint16_t tok_s[kChunk / 2 + 8];
  uint16_t tok_e[kChunk / 2 + 8];
  uint64_t wbits[(kPreMargin + kChunk + kPostMargin) / 64 + 2];
  uint32_t rcnt[64];
  uint32_t rcur[64];
  uint32_t scan[8];
  uint32_t len, flags, nu, pad;
  uint8_t lut[128];
  alignas(16) uint8_t text[kPreMargin + kChunk + kPostMargin + 64];
};

__global__ void __launch_bounds__(256) k_tokenize_long(BuildParams p) {
  __shared__ LongSmem sm;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 128; i += 256) sm.lut[i] = wb_class(i);
  if (tid < 64) { sm.rcnt[tid] = 0; sm.rcur[tid] = 0; }
  if (tid == 0) { sm.len = 0; sm.flags = 0; sm.nu = 0; }
  __syncthreads();
  const uint32_t n_long = *p.long_count;
  uint64_t *keys = p.lt_keys + (size_t)blockIdx.x * 2 * (1ull << p.lt_slots_log2);
  uint32_t *cnt = p.lt_cnt + (size_t)blockIdx.x * (1ull << p.lt_slots_log2);
  uint32_t *gsl = p.lt_g + (size_t)blockIdx.x * (1ull << p.lt_slots_log2);
  uint64_t *tpos = p.lt_pos + (size_t)blockIdx.x * (1ull << p.lt_slots_log2);
  unsigned long long my_doc_count = 0, my_ttf = 0, my_nnz = 0;

  for (uint32_t li = blockIdx.x; li < n_long; li += gridDim.x) {
    const uint32_t d = p.long_list[li];
    const uint64_t src = p.live_map ? p.live_map[d] : d;
    const uint64_t s0 = p.offsets[src], s1 = p.offsets[src + 1];
    const uint64_t L = s1 - s0;
    // table size: >= 2x the token upper bound (L/2 + 1), capped
    uint32_t lg = 10;
    while (lg < p.lt_slots_log2 && (1ull << lg) < L + 2) lg++;
    const uint32_t T = 1u << lg, mask = T - 1;
    for (uint32_t i = tid; i < T; i += 256) { keys[2 * i] = 0; keys[2 * i + 1] = 0; cnt[i] = 0; tpos[i] = 0; }
    __syncthreads();
    uint32_t my_len = 0;
    bool bad = false;
    for (uint64_t cs = 0; cs < L; cs += kChunk) {
      const uint64_t ce = cs + kChunk < L ? cs + kChunk : L;
      const uint64_t wlo = cs >= kPreMargin ? cs - kPreMargin : 0;
      const uint64_t whi = ce + kPostMargin < L ? ce + kPostMargin : L;
      const uint32_t wlen = (uint32_t)(whi - wlo);
      uint32_t shift;
      stage_bytes(sm.text, p.text + s0 + wlo, wlen, &shift);
      __syncthreads();
      const uint32_t hi_b = shift + wlen;
      if (phase_wordbits(sm.text, shift, hi_b, sm.wbits, &sm.flags)) { bad = true; break; }
      const uint32_t ntok = phase_token_spans(sm.wbits, hi_b, shift + (uint32_t)(cs - wlo),
                                              shift + (uint32_t)(ce - wlo), sm.tok_s, sm.tok_e, kChunk / 2 + 8, sm.scan);
      for (uint32_t i = tid; i < ntok; i += 256) {
        const uint32_t s = sm.tok_s[i], e = sm.tok_e[i];
        if (e - s > kMaxTokenLen) { atomicOr(&sm.flags, 8u); continue; }   // cut by the Unicode scanner
        uint64_t lo, hi;
        bool valid;
        token_key(sm.text, s, e, &lo, &hi, &valid, p.hash_seed);
        if (!valid) continue;
        my_len++;
        const uint64_t occ = dict_ref_word(wlo + (s - shift), e - s);
        if (gtable_insert(keys, cnt, tpos, mask, lo, hi, occ, p.text + s0, p.err, d) == kInvalidSlot)
          atomicOr(&sm.flags, 4u);
      }
      __syncthreads();
    }
    if (bad || (sm.flags & 8u)) {
      // General phase (unicode_scan.h): a non-ASCII byte or a token of more
      // than 255 chars.  Reset the table and rescan the whole document with
      // the full-Unicode scanner: thread t takes the tokens starting in its
      // slice of the document, slices cut just after ASCII class-OTHER bytes
      // (the scan restarts there in the start state).
      for (uint32_t i = tid; i < T; i += 256) { keys[2 * i] = 0; keys[2 * i + 1] = 0; cnt[i] = 0; tpos[i] = 0; }
      __syncthreads();
      my_len = 0;
      const uint8_t *doc = p.text + s0;
      const uint64_t seg = L / 256 + 64;
      auto slice = [&](uint64_t t) -> uint64_t {
        if (t == 0) return 0;
        uint64_t q = t * seg;
        if (q >= L) return L;
        while (q < L && !uc_split_byte(doc[q - 1])) q++;
        return q;
      };
      uint64_t pos = slice(tid);
      const uint64_t stop = slice(tid + 1);
      uint64_t ts, te, lo, hi;
      bool ubad = false;
      while (uc_next_token(doc, L, &pos, stop, &ts, &te, &lo, &hi, &ubad, p.hash_seed)) {
        my_len++;
        if (gtable_insert(keys, cnt, tpos, mask, lo, hi, dict_ref_word(ts, (uint32_t)(te - ts)), doc, p.err, d) ==
            kInvalidSlot)
          atomicOr(&sm.flags, 4u);
      }
      if (ubad) atomicOr(&sm.flags, 16u);
      __syncthreads();
      bad = (sm.flags & 16u) != 0;
    }
    if (bad) {                                   // malformed UTF-8: indexed empty and listed
      if (tid == 0) {                            // (Files.readString throws; the host supplies the
        p.bad_list[atomicAdd(p.bad_count, 1u)] = d;   // extracted text, Worker.java:199-211)
        p.doc_len[d] = 0; p.doc_nuniq[d] = 0; p.doc_norm[d] = 0;
        for (uint32_t r = 0; r < p.n_ranges; r++) p.rsplit[(uint64_t)d * p.n_ranges + r] = 0;
        sm.flags = 0;
      }
      __syncthreads();
      continue;
    }
    if (sm.flags & 4u) set_err(p.err, kErrLongScratch, d);
    atomicAdd(&sm.len, my_len);
    // emission: dictionary lookup + range counts
    uint32_t my_nu = 0;
    for (uint32_t sb = 0; sb < T; sb += 256) {
      const uint32_t s = sb + tid;
      uint64_t lo = 0, hi = 0;
      if (s < T) {
        lo = __hip_atomic_load(keys + 2 * (size_t)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hi = __hip_atomic_load(keys + 2 * (size_t)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const bool act = lo != 0;
      uint64_t mine = 0;
      if (act && (lo & kLoHashed)) {
        const uint64_t r = __hip_atomic_load(tpos + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mine = dict_ref_word(s0 + dict_ref_off(r), dict_ref_len(r));       // document-relative -> corpus offset
      }
      bool cl;
      uint32_t g = dict_find_or_insert(p.dict, p.cap_mask, act ? lo : 1, act ? hi : kKeyValid, act, &mine, &cl);
      if (act && (lo & kLoHashed) && !cl && g != kInvalidSlot) dict_verify(p, g, mine, d);
      if (act) {
        if (g == kInvalidSlot) { set_err(p.err, kErrCapacity, d); g = 0; }
        gsl[s] = g;
        atomicAdd(&sm.rcnt[g >> p.range_shift], 1u);
        my_nu++;
      }
    }
    atomicAdd(&sm.nu, my_nu);
    __syncthreads();
    if (tid == 0) {
      uint32_t run = 0;
      for (uint32_t r = 0; r < p.n_ranges; r++) {
        const uint32_t c = sm.rcnt[r];
        sm.rcur[r] = run;
        run += c;
        p.rsplit[(uint64_t)d * p.n_ranges + r] = run;
        sm.rcnt[r] = 0;
      }
      const uint32_t len = sm.len;
      p.doc_len[d] = len;
      p.doc_nuniq[d] = sm.nu;
      p.doc_norm[d] = (uint8_t)int_to_byte4(len);
      my_doc_count += len > 0;
      my_ttf += len;
      my_nnz += sm.nu;
    }
    __syncthreads();
    const uint64_t base = csr_row_base(p.offsets, src);
    for (uint32_t s = tid; s < T; s += 256) {
      if (__hip_atomic_load(keys + 2 * (size_t)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) continue;
      const uint32_t g = gsl[s];
      const uint32_t pos = atomicAdd(&sm.rcur[g >> p.range_shift], 1u);
      csr_put(p, base + pos, g, __hip_atomic_load(cnt + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), d);
    }
    __syncthreads();
    if (tid == 0) { sm.len = 0; sm.flags = 0; sm.nu = 0; }
    __syncthreads();
  }
  if (tid == 0) {
    atomicAdd(&p.stats[0], my_doc_count);
    atomicAdd(&p.stats[1], my_ttf);
    atomicAdd(&p.stats[2], my_nnz);
  }
}

// ---------------------------------------------------------------------------
// Inversion.

__device__ __forceinline__ void doc_segment(const PostingParams &p, uint64_t d, uint32_t r, uint64_t *base,
                                            uint32_t *lo, uint32_t *hi) {
  const uint64_t src = p.live_map ? p.live_map[d] : d;
  *base = csr_row_base(p.offsets, src);
  *lo = r ? p.rsplit[d * p.n_ranges + r - 1] : 0;
  *hi = p.rsplit[d * p.n_ranges + r];
}

// Documents per wave in flight in the inversion kernels: each wave walks
// kInvDocs documents' segments together so their loads overlap, and issues
// the next group's segment loads before the current group's LDS atomics and
// stores (gfx9 counts stores in vmcnt: waiting for loads issued after a
// store would also wait for the store).
#ifndef TFIDF_INV_DOCS
#define TFIDF_INV_DOCS 8
#endif
constexpr int kInvDocs = TFIDF_INV_DOCS;   // A/B: -DTFIDF_INV_DOCS=16

struct InvGroup {               // wave-uniform
  uint64_t base[kInvDocs];
  uint32_t lo[kInvDocs], hi[kInvDocs], nrm[kInvDocs];
  uint32_t maxn;
};

// Group metadata, loaded lane-parallel (lane j < kInvDocs fetches document j:
// one round trip for the whole group instead of a dependent scalar chain per
// document) and broadcast with readlane.
__device__ __forceinline__ InvGroup inv_group(const PostingParams &p, uint64_t dd, uint64_t d1, uint32_t stride,
                                              uint32_t r, bool with_norm) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t d = dd + (uint64_t)stride * (lane & (kInvDocs - 1));
  const bool ok = lane < (uint32_t)kInvDocs && d < d1;
  uint64_t base = 0;
  uint32_t lo = 0, hi = 0, nrm = 0;
  if (ok) {
    const uint64_t src = p.live_map ? p.live_map[d] : d;
    base = csr_row_base(p.offsets, src);
    lo = r ? p.rsplit[d * p.n_ranges + r - 1] : 0;
    hi = p.rsplit[d * p.n_ranges + r];
    if (with_norm) nrm = p.doc_norm[d];
  }
  InvGroup g;
  g.maxn = 0;
#pragma unroll
  for (int j = 0; j < kInvDocs; j++) {
    g.base[j] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(base >> 32), j) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, j);
    g.lo[j] = (uint32_t)__builtin_amdgcn_readlane((int)lo, j);
    g.hi[j] = (uint32_t)__builtin_amdgcn_readlane((int)hi, j);
    g.nrm[j] = (uint32_t)__builtin_amdgcn_readlane((int)nrm, j);
    g.maxn = max(g.maxn, g.hi[j] - g.lo[j]);
  }
  return g;
}

// packed CSR words off of the group's documents' segments (0 past a segment)
__device__ __forceinline__ void inv_load(const PostingParams &p, const InvGroup &g, uint32_t off, uint32_t *c) {
#pragma unroll
  for (int j = 0; j < kInvDocs; j++) {
    const bool in = g.lo[j] + off < g.hi[j];
    c[j] = in ? p.csr[g.base[j] + g.lo[j] + off] : 0u;
  }
}

// (block, range) tile of a 1-D grid of tiles_grid() workgroups: the R tiles
// of a block get workgroup ids congruent mod 8, dispatched together, so they
// run on one XCD and the CSR lines their row segments share come from that
// XCD's L2 instead of being fetched once per range (dispatch order is only a
// placement hint: correctness never depends on it).
__device__ __forceinline__ bool tile_of(uint32_t w, uint32_t n_blocks, uint32_t R, uint32_t *b, uint32_t *r) {
  const uint32_t g = w / (8 * R), rem = w - g * 8 * R;
  *r = rem >> 3;
  *b = g * 8 + (rem & 7);
  return *b < n_blocks;
}
static uint32_t tiles_grid(uint32_t n_blocks, uint32_t R) { return (n_blocks + 7) / 8 * 8 * R; }

// one workgroup (1024 threads) per (block, range) tile (tile_of): LDS
// histogram of the range's 65536 slots in 16-bit counters (two per word; a
// block's count of one slot is at most kBlockDocs = 8192), 128 KiB.  Wave w
// handles documents d0 + w + 16 (kInvDocs i + j), j < kInvDocs.  The counts
// of the range's occupied slots are written at their columns (col_rank), so
// the count table follows the vocabulary, not the dictionary's probe table.
__global__ void __launch_bounds__(1024) k_df_partial(PostingParams p) {
  extern __shared__ uint32_t hist[];
  uint32_t b, r;
  if (!tile_of(blockIdx.x, p.n_blocks, p.n_ranges, &b, &r)) return;
  const uint32_t RS = 1u << p.range_shift;
  for (uint32_t i = threadIdx.x; i < RS / 2; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const uint64_t d0 = (uint64_t)b * kBlockDocs;
  const uint64_t d1 = d0 + kBlockDocs < p.n_docs ? d0 + kBlockDocs : p.n_docs;
  const uint32_t lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t rmask = RS - 1;
  const uint64_t step = (uint64_t)nw * kInvDocs;
  uint64_t dd = d0 + wid;
  InvGroup cur = inv_group(p, dd, d1, nw, r, false);
  uint32_t c[kInvDocs];
  if (dd < d1) inv_load(p, cur, lane, c);
  auto count = [&](uint32_t e) __attribute__((always_inline)) {
    const uint32_t sl = e & rmask;
    atomicAdd(&hist[sl >> 1], 1u << ((sl & 1u) << 4));
  };
  while (dd < d1) {
    const uint64_t dn = dd + step;
    const InvGroup nxt = inv_group(p, dn, d1, nw, r, false);
    uint32_t cn[kInvDocs];
    if (dn < d1) inv_load(p, nxt, lane, cn);                       // next group in flight
#pragma unroll
    for (int j = 0; j < kInvDocs; j++)
      if (c[j]) count(c[j]);
    for (uint32_t off = lane + 64; off < cur.maxn; off += 64) {     // segments longer than 64
      inv_load(p, cur, off, c);
#pragma unroll
      for (int j = 0; j < kInvDocs; j++)
        if (c[j]) count(c[j]);
    }
    cur = nxt;
#pragma unroll
    for (int j = 0; j < kInvDocs; j++) c[j] = cn[j];
    dd = dn;
  }
  __syncthreads();
  // occupied slots of the range -> their columns (a word's slots hold
  // consecutive columns from its prefix count)
  uint32_t *out = p.blk + (size_t)b * p.NC;
  const uint32_t w0 = (r << p.range_shift) >> 5;
  for (uint32_t w = threadIdx.x; w < (RS >> 5); w += blockDim.x) {
    const uint2 e = p.crank[w0 + w];
    uint32_t bits = e.x, col = e.y;
    while (bits) {
      const uint32_t sl = 32 * w + (uint32_t)__builtin_ctz(bits);
      bits &= bits - 1;
      out[col++] = (hist[sl >> 1] >> ((sl & 1u) << 4)) & 0xFFFFu;
    }
  }
}

// per column: df = sum of the per-block counts (row n_blocks).
__global__ void __launch_bounds__(256) k_df_sum(PostingParams p) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.NC) return;
  uint32_t run = 0;
  for (uint32_t b = 0; b < p.n_blocks; b++) run += p.blk[(size_t)b * p.NC + t];
  p.blk[(size_t)p.n_blocks * p.NC + t] = run;
}

// per block row: exclusive scan over columns in place (one workgroup per row);
// the row total goes to bbase[b + 1] (turned into bases by k_block_scan).
// Tiles of 16384 columns: each thread loads 16 consecutive counts with four
// 16 B loads (coalesced across the workgroup), scans them in registers, and a
// workgroup scan of the 1024 thread totals gives the offsets.
__global__ void __launch_bounds__(1024) k_row_scan(PostingParams p) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry_sh;
  uint32_t *row = p.blk + (size_t)blockIdx.x * p.NC;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) carry_sh = 0;
  __syncthreads();
  for (uint32_t t0 = 0; t0 < p.NC; t0 += 16384) {
    const uint32_t i0 = t0 + tid * 16;
    uint32_t v[16];
    if (i0 + 16 <= p.NC) {
      const uint4 *src = reinterpret_cast<const uint4 *>(row + i0);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint4 x = src[q];
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; q++) v[q] = (i0 + q < p.NC) ? row[i0 + q] : 0u;
    }
    uint32_t tot = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) tot += v[q];
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t base = carry_sh, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
      const uint32_t sw = wsum[w];
      if (w < wid) base += sw;
      all += sw;
    }
    base += x - tot;
    __syncthreads();
    if (tid == 0) carry_sh += all;
    uint32_t run = base;
    uint32_t o[16];
#pragma unroll
    for (int q = 0; q < 16; q++) { o[q] = run; run += v[q]; }
    if (i0 + 16 <= p.NC) {
      uint4 *dst = reinterpret_cast<uint4 *>(row + i0);
#pragma unroll
      for (int q = 0; q < 4; q++) dst[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
    } else {
#pragma unroll
      for (int q = 0; q < 16; q++)
        if (i0 + q < p.NC) row[i0 + q] = o[q];
    }
    __syncthreads();
  }
  if (tid == 0) p.bbase[blockIdx.x + 1] = carry_sh;
}

// Inversion in two passes so that every store stream stays L2-resident.
// A (block, range) tile's postings span ~10 k term regions: storing each
// posting straight to its final column keeps that many partial lines open per
// workgroup and writes back ~3x the bytes.  Instead:
//   k_scatter_part : per tile, each posting is appended to one of the tile's
//                    64 sub-range streams (kSubSlots dictionary slots each) in
//                    a temporary buffer laid out exactly like the postings
//                    (stream k's region = the final region of its slots'
//                    columns, from blk), one 32-bit word doc_local(13) |
//                    slot_low(10) | tf(9); tf >= 511 is stored as 511 and
//                    re-read from the CSR row in pass 2, the norm is re-read
//                    from doc_norm there;
//   k_scatter_sort : per stream, LDS cursor per slot, final postings written
//                    inside the stream's own region.
constexpr uint32_t kSubBits = 10;
constexpr uint32_t kSubSlots = 1u << kSubBits;
constexpr uint32_t kTmpTfShift = 13 + kSubBits;              // temp word: doc_local(13) | slot_low | tf(9)
constexpr uint32_t kTmpTfEsc = (1u << (32 - kTmpTfShift)) - 1; // tf field value meaning "tf >= this: see the CSR"
constexpr uint32_t kPartStreams = kRangeSlots / kSubSlots;  // 64
static_assert(kTmpTfShift <= 23 && kPartStreams == 64, "temp word layout");

__device__ __forceinline__ void part_entries(const PostingParams &p, uint32_t *bcur, uint32_t rmask, uint64_t bb,
                                             const InvGroup &g, uint64_t dd, uint32_t d0l, uint32_t stride,
                                             const uint32_t *c) {
  const uint32_t lane = threadIdx.x & 63;
  constexpr uint32_t kNoop = kPartStreams;                    // idle lanes bump a spare cursor
#pragma unroll
  for (int j = 0; j < kInvDocs; j++) {
    const bool in = c[j] != 0;
    if (!__any(in)) continue;                                 // wave-uniform
    const uint32_t sl = c[j] & rmask;
    const uint32_t dl = (uint32_t)(dd + (uint64_t)stride * j) - d0l;
    const uint32_t tf = csr_tf_field(c[j], p.range_shift);
    const uint32_t val = dl | ((sl & (kSubSlots - 1)) << 13) | (min(tf, kTmpTfEsc) << kTmpTfShift);
    const uint32_t pos = cursor_bump<kRangeBits - kSubBits + 1>(bcur, in ? sl >> kSubBits : kNoop, lane);
    if (in) p.post_tmp[bb + pos] = val;
  }
}

// Workgroup-wide staging (round 5).  All the workgroup's waves take their next
// document group together (a round: nw * kInvDocs documents, up to 8 192
// entries); the round's entries are counting-sorted by sub-range stream in LDS
// and stored stream run by stream run, ~16x longer runs than wave-local
// staging (one to two lines per store instruction instead of ~13).
__global__ void __launch_bounds__(1024) k_scatter_part(PostingParams p) {
  __shared__ uint32_t bcur[kPartStreams + 1];
  __shared__ uint32_t cnt[kPartStreams], soff[kPartStreams], gb[kPartStreams], tot_sh;
  __shared__ uint32_t stage[16 * kInvDocs * 64];
  __shared__ uint8_t sid[16 * kInvDocs * 64];
  const uint32_t lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint32_t b, r;
  if (!tile_of(blockIdx.x, p.n_blocks, p.n_ranges, &b, &r)) return;
  const uint32_t RS = 1u << p.range_shift, rmask = RS - 1;
  const uint32_t nsub = RS > kSubSlots ? RS / kSubSlots : 1u;
  const uint32_t *row = p.blk + (size_t)b * p.NC;
  if (threadIdx.x < nsub) {
    // stream k's region starts at the column of its first occupied slot (=
    // the occupied slots before it, col_rank); an empty stream is never bumped
    const uint32_t c0 = p.crank[((r << p.range_shift) + threadIdx.x * kSubSlots) >> 5].y;
    bcur[threadIdx.x] = c0 < p.NC ? row[c0] : 0u;
  }
  if (threadIdx.x < kPartStreams) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t bb = p.bbase[b];
  const uint64_t d0 = (uint64_t)b * kBlockDocs;
  const uint64_t d1 = d0 + kBlockDocs < p.n_docs ? d0 + kBlockDocs : p.n_docs;
  const uint64_t step = (uint64_t)nw * kInvDocs;
  const uint32_t rounds = (uint32_t)((d1 - d0 + step - 1) / step);   // workgroup-uniform
  uint64_t dd = d0 + wid;
  InvGroup g = inv_group(p, dd, d1, nw, r, false);
  uint32_t c[kInvDocs];
  if (dd < d1) inv_load(p, g, lane, c);
  else
#pragma unroll
    for (int j = 0; j < kInvDocs; j++) c[j] = 0;
  for (uint32_t k = 0; k < rounds; k++) {
    const uint64_t dn = dd + step;
    const InvGroup gn = inv_group(p, dn, d1, nw, r, false);
    uint32_t cn[kInvDocs];
#pragma unroll
    for (int j = 0; j < kInvDocs; j++) cn[j] = 0;
    if (dn < d1) inv_load(p, gn, lane, cn);                       // next group in flight
    uint32_t val[kInvDocs], rank[kInvDocs], sj[kInvDocs];
#pragma unroll
    for (int j = 0; j < kInvDocs; j++) {
      const uint32_t sl = c[j] & rmask;
      sj[j] = sl >> kSubBits;
      const uint32_t dl = (uint32_t)(dd + (uint64_t)nw * j - d0);
      const uint32_t tf = csr_tf_field(c[j], p.range_shift);
      val[j] = dl | ((sl & (kSubSlots - 1)) << 13) | (min(tf, kTmpTfEsc) << kTmpTfShift);
      rank[j] = c[j] != 0 ? atomicAdd(&cnt[sj[j]], 1u) : 0u;
    }
    __syncthreads();                                              // the round's counts are complete
    if (wid == 0) {
      const uint32_t n = cnt[lane];
      const uint32_t incl = wave_incl_add(n);
      soff[lane] = incl - n;
      gb[lane] = n ? atomicAdd(&bcur[lane], n) : 0u;
      cnt[lane] = 0;
      if (lane == 63) tot_sh = incl;
    }
    __syncthreads();                                              // offsets known
#pragma unroll
    for (int j = 0; j < kInvDocs; j++)
      if (c[j] != 0) {
        const uint32_t at = soff[sj[j]] + rank[j];
        stage[at] = val[j];
        sid[at] = (uint8_t)sj[j];
      }
    __syncthreads();                                              // the round's entries are staged
    const uint32_t T = tot_sh;
    for (uint32_t ti = threadIdx.x; ti < T; ti += blockDim.x) {
      const uint32_t st = sid[ti];
      p.post_tmp[bb + gb[st] + (ti - soff[st])] = stage[ti];
    }
    for (uint32_t off = lane + 64; off < g.maxn; off += 64) {    // segments longer than 64
      inv_load(p, g, off, c);
      part_entries(p, bcur, rmask, bb, g, dd, (uint32_t)d0, nw, c);
    }
    g = gn;
#pragma unroll
    for (int j = 0; j < kInvDocs; j++) c[j] = cn[j];
    dd = dn;
    // the next round's counts go to cnt (reset above); its stage / soff / gb
    // writes come after its first barrier, when every thread has left this
    // round's store loop
  }
}

// tf of (doc, slot) from the document's CSR row segment of range r (the
// escape path of the 9-bit temp tf field; rare)
__device__ uint32_t csr_tf_of(const PostingParams &p, uint64_t d, uint32_t r, uint32_t slot) {
  uint64_t base;
  uint32_t lo, hi;
  doc_segment(p, d, r, &base, &lo, &hi);
  const uint32_t local = csr_local(slot, p.range_shift), esc = csr_esc_value(p.range_shift);
  for (uint32_t i = lo; i < hi; i++) {
    const uint32_t e = p.csr[base + i];
    if (csr_local(e, p.range_shift) == local) {
      const uint32_t f = csr_tf_field(e, p.range_shift);
      return f == esc ? csr_esc_tf(p.csr_esc, p.n_esc, base + i) : f;
    }
  }
  return 0;
}

// grid (n_blocks, n_ranges, streams per range / sort_spw), 512 threads; a
// workgroup takes sort_spw = 4 streams in turn, so few streams per CU are open
// at a time and the regions being written stay L2-resident (cfg-2 inversion:
// one stream per 1024-thread workgroup 3.11 ms, 8 per 1024 2.87, 4 per 512 2.52)
// Round 5: a stream of at most kSortStage entries is assembled in LDS and
// written out contiguous (its region is [lo, hi) of the block's postings);
// scattered 4-byte global stores only for larger streams (4 096 / 6 144 /
// 8 192 / 16 384 measured 2.03 / 1.93 / 1.85 / 1.97 ms scatter at cfg 2).
constexpr uint32_t kSortStage = 8192;
constexpr uint32_t kSortMaxSpw = 8;
__global__ void __launch_bounds__(1024) k_scatter_sort(PostingParams p) {
  __shared__ uint32_t cur[kSubSlots + 1];                   // + no-op cursor for idle lanes
  __shared__ uint32_t ostage[kSortStage];
  __shared__ uint8_t bnorm[kBlockDocs];                     // the block's norm bytes: an LDS read per entry
                                                            // instead of a global load that waits on the temp word
  __shared__ uint2 wk[kSortMaxSpw * (kSubSlots / 32) + 1];  // the streams' column ranks (col_rank)
  const uint32_t b = blockIdx.x, r = blockIdx.y;
  const uint32_t RS = 1u << p.range_shift;
  const uint32_t BS = RS < kSubSlots ? RS : kSubSlots;
  const uint32_t nsub = RS / BS;
  const uint32_t k0 = blockIdx.z * p.sort_spw, k1 = min(nsub, k0 + p.sort_spw);
  if (k0 >= k1) return;
  const uint32_t *row = p.blk + (size_t)b * p.NC;
  const uint64_t bb = p.bbase[b];
  const uint32_t btot = (uint32_t)(p.bbase[b + 1] - bb);
  const uint32_t d0 = b * kBlockDocs;
  const uint32_t sw0 = ((r << p.range_shift) + k0 * BS) >> 5, nwk = (k1 - k0) * BS / 32 + 1;
  for (uint32_t i = threadIdx.x; i < nwk; i += blockDim.x) wk[i] = p.crank[sw0 + i];   // (+1: the sentinel / next word)
  {
    const uint32_t nd = (uint32_t)min((uint64_t)kBlockDocs, p.n_docs - d0);
    for (uint32_t i = threadIdx.x * 16; i < nd; i += blockDim.x * 16) {
      if (i + 16 <= nd) {
        *reinterpret_cast<uint4 *>(&bnorm[i]) = *reinterpret_cast<const uint4 *>(p.doc_norm + d0 + i);
      } else {
        for (uint32_t j = i; j < nd; j++) bnorm[j] = p.doc_norm[d0 + j];
      }
    }
  }
  __syncthreads();
  for (uint32_t k = k0; k < k1; k++) {
    // the stream's slots s0 .. s0 + BS - 1 hold columns c0 .. c1 - 1
    const uint32_t s0 = (r << p.range_shift) + k * BS;
    const uint2 *kw = wk + (k - k0) * (BS / 32);
    const uint32_t c0 = kw[0].y, c1 = kw[BS / 32].y;
    if (c0 == c1) continue;                                   // workgroup-uniform: no occupied slot
    for (uint32_t i = threadIdx.x; i < BS; i += blockDim.x) {
      const uint2 e = kw[i >> 5];
      const uint32_t bit = 1u << (i & 31u);
      if (e.x & bit) cur[i] = row[e.y + __popc(e.x & (bit - 1u))];
    }
    const uint32_t lo = row[c0];
    const uint32_t hi = c1 < p.NC ? row[c1] : btot;
    const bool staged = hi - lo <= kSortStage;                // workgroup-uniform
    __syncthreads();
    constexpr int U = 8;              // entries per thread in flight (8: a ~5 k-entry stream in one round; round 5 with
                                      // staging + plain atomics: 4 / 8 / 12 / 16 = 1.91 / 1.86 / 1.84 / 1.84 ms scatter)
    for (uint32_t e0 = lo; e0 < hi; e0 += U * blockDim.x) {   // uniform trip count: all lanes ballot
      uint32_t x[U], nrm[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t e = e0 + u * blockDim.x + threadIdx.x;
        x[u] = e < hi ? p.post_tmp[bb + e] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t e = e0 + u * blockDim.x + threadIdx.x;
        nrm[u] = e < hi ? bnorm[x[u] & (kBlockDocs - 1)] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t e = e0 + u * blockDim.x + threadIdx.x;
        if (__all(e >= hi)) break;
        const bool in = e < hi;
        const uint32_t sl = in ? (x[u] >> 13) & (kSubSlots - 1) : kSubSlots;   // kSubSlots: no-op key
        // plain LDS atomics on the slot cursors (order inside a (block, slot)
        // segment is free); with the LDS-staged output they beat the wave
        // peer-mask bump (10 ballots per entry): scatter 2.34 -> 1.99 ms at cfg 2
        // (without staging the peer-mask bump was 4 % faster)
        const uint32_t pos = atomicAdd(&cur[sl], 1u);
        const uint32_t doc = d0 + (x[u] & (kBlockDocs - 1));
        uint32_t tf = x[u] >> kTmpTfShift;
        if (in && tf == kTmpTfEsc) tf = csr_tf_of(p, doc, r, s0 + sl);                // rare: tf >= 511
        if (in) {
          const uint32_t w = post_word(x[u] & (kBlockDocs - 1), tf, nrm[u]);
          if (staged) ostage[pos - lo] = w;
          else p.post[bb + pos] = w;
          if (tf >= kPostTfEsc) {                                                 // rare: tf >= 2047
            const uint32_t at = atomicAdd(p.post_esc_count, 1u);
            if (at < p.post_esc_cap) p.post_esc[at] = ((bb + pos) << 24) | tf;
          }
        }
      }
    }
    __syncthreads();                                      // the stream's words are in ostage
    if (staged)
      for (uint32_t i = threadIdx.x; i < hi - lo; i += blockDim.x) p.post[bb + lo + i] = ostage[i];
    __syncthreads();                                      // cursors and ostage reused by the next stream
  }
}

// block totals in bbase[b + 1] -> block bases, in place (one workgroup; every
// total of a round is read before the barrier, written after it)
__global__ void __launch_bounds__(1024) k_block_scan(PostingParams p) {
  __shared__ uint64_t wsum[16];
  const uint32_t B = p.n_blocks;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint64_t carry = 0;
  for (uint32_t i0 = 0; i0 < B; i0 += 1024) {
    const uint32_t i = i0 + tid;
    const uint64_t v = i < B ? p.bbase[i + 1] : 0ull;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint64_t base = carry, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
      const uint64_t s = wsum[w];
      if (w < wid) base += s;
      all += s;
    }
    __syncthreads();
    if (i < B) p.bbase[i + 1] = base + x;            // inclusive = the next block's base
    carry += all;
  }
  if (tid == 0) p.bbase[0] = 0;
}

// Hashed-key checks deferred by dict_verify (the slot's reference occurrence
// was not visible yet): every reference is final after the tokenizers.
__global__ void __launch_bounds__(256) k_verify_deferred(BuildParams p) {
  const uint32_t n = min(*p.verify_count, p.verify_cap);
  const uint64_t *ref = p.dict + 2 * ((size_t)p.cap_mask + 1);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t slot = (uint32_t)p.verify_defer[2 * (size_t)i];
    const uint64_t mine = p.verify_defer[2 * (size_t)i + 1], r = ref[slot];
    if (r == mine) continue;
    if (r == 0 || !uc_same_term(p.text + dict_ref_off(r), dict_ref_len(r), p.text + dict_ref_off(mine),
                                dict_ref_len(mine)))
      set_build_err(p.err, kErrCollision, 0);
  }
}

// ---------------------------------------------------------------------------
// launchers

hipError_t launch_verify_deferred(const BuildParams &p, hipStream_t s) {
  hipLaunchKernelGGL(k_verify_deferred, dim3(64), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_tokenize_wave(const BuildParams &p, int grid, hipStream_t s) {
#ifndef TFIDF_G4_BITS
#define TFIDF_G4_BITS 21
#endif
  const bool g4 = (uint64_t)p.cap_mask + 1 >= (1ull << TFIDF_G4_BITS);   // dictionary beyond L2: 4-slot probe groups
  if (p.pack > 1) {
    if (g4) hipLaunchKernelGGL((k_tokenize_wave<true, true>), dim3(grid), dim3(64), 0, s, p);
    else hipLaunchKernelGGL((k_tokenize_wave<true, false>), dim3(grid), dim3(64), 0, s, p);
  } else {
    if (g4) hipLaunchKernelGGL((k_tokenize_wave<false, true>), dim3(grid), dim3(64), 0, s, p);
    else hipLaunchKernelGGL((k_tokenize_wave<false, false>), dim3(grid), dim3(64), 0, s, p);
  }
  return hipGetLastError();
}
// The flagged (non-ASCII) documents by the wave rules where they allow
// (k_tokenize_wave<UNI>); before k_tokenize_uwave, which takes the rest.
hipError_t launch_tokenize_wave_uni(const BuildParams &p, int grid, hipStream_t s) {
  const bool g4 = (uint64_t)p.cap_mask + 1 >= (1ull << TFIDF_G4_BITS);
  if (g4) hipLaunchKernelGGL((k_tokenize_wave<false, true, true>), dim3(grid), dim3(64), 0, s, p);
  else hipLaunchKernelGGL((k_tokenize_wave<false, false, true>), dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_tokenize_chunks(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_chunk<false>, dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}
// The units k_tokenize_chunk flagged for non-ASCII text, by the wave rules
// where they allow (k_tokenize_chunk<UNI>); before k_tokenize_uchunk.
hipError_t launch_tokenize_chunks_uni(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_chunk<true>, dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_long_rows(const BuildParams &p, uint32_t n_docs, hipStream_t s) {
  static std::atomic<uint64_t> big{0};
  allow_dyn_lds((const void *)k_long_rows, 4 * kLrWin, big);
  const uint32_t C = p.cap_mask + 1;
  hipLaunchKernelGGL(k_long_rows, dim3(n_docs), dim3(kLrThreads), (C < kLrWin ? C : kLrWin) * 4, s, p);
  return hipGetLastError();
}
hipError_t launch_tokenize_long(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_long, dim3(grid), dim3(256), 0, s, p);
  return hipGetLastError();
}
static void allow_big_lds() {
  static std::atomic<uint64_t> done{0};
  allow_dyn_lds((const void *)k_df_partial, 2 << kRangeBits, done);
}

hipError_t launch_df_partial(const PostingParams &p, hipStream_t s) {
  allow_big_lds();
  const size_t lds = (size_t)2 << p.range_shift;             // 16-bit counters
  hipLaunchKernelGGL(k_df_partial, dim3(tiles_grid(p.n_blocks, p.n_ranges)), dim3(1024), lds, s, p);
  return hipGetLastError();
}
hipError_t launch_df_sum(const PostingParams &p, hipStream_t s) {
  if (p.NC == 0) return hipSuccess;
  hipLaunchKernelGGL(k_df_sum, dim3((p.NC + 255) / 256), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_row_scan(const PostingParams &p, hipStream_t s) {
  hipLaunchKernelGGL(k_row_scan, dim3(p.n_blocks), dim3(1024), 0, s, p);
  return hipGetLastError();
}
// number of nonzero entries of a[0, n) (occupied dictionary slots): one
// ballot per wave, one atomic per wave
__global__ void __launch_bounds__(256) k_count_nonzero(const uint64_t *a, uint32_t n, unsigned long long *out) {
  uint32_t c = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint64_t m = __ballot(a[i] != 0);
    c += (uint32_t)__popcll(m);
  }
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}
hipError_t launch_count_nonzero(const uint64_t *a, uint32_t n, unsigned long long *out, hipStream_t s) {
  const uint32_t grid = std::max(1u, std::min((n + 255) / 256, 2048u));
  hipLaunchKernelGGL(k_count_nonzero, dim3(grid), dim3(256), 0, s, a, n, out);
  return hipGetLastError();
}
// ---- columns of the block-major inversion (round 6).  The dictionary is a
// probe table (load 0.2-0.4: fewer dependent probe rounds in the tokenizer);
// the count table, its scans and the postings are indexed by the rank of an
// occupied slot ("column", 0 .. num_terms - 1), so their size follows the
// vocabulary, not the probe table.  crank[w] = {occupancy bits of slots 32 w
// .. 32 w + 31, occupied slots before 32 w}; crank[C / 32] = {0, num_terms}.
// Column of occupied slot s: crank[s / 32].y + popc(bits below s).
__global__ void __launch_bounds__(256) k_crank_bits(const uint64_t *lo, uint32_t C, uint2 *crank) {
  const uint32_t s0 = (blockIdx.x * blockDim.x + threadIdx.x) & ~63u, lane = threadIdx.x & 63;
  if (s0 >= C) return;                                        // wave-uniform (C is a multiple of 64)
  const uint64_t m = __ballot(lo[s0 + lane] != 0);
  if (lane < 2) crank[(s0 >> 5) + lane] = make_uint2(lane ? (uint32_t)(m >> 32) : (uint32_t)m, 0u);
}
// exclusive scan of the words' popcounts (one workgroup; 16 words per thread
// per tile, as k_row_scan); the total = columns
__global__ void __launch_bounds__(1024) k_crank_scan(uint2 *crank, uint32_t W, unsigned long long *n_cols) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry_sh;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) carry_sh = 0;
  __syncthreads();
  for (uint32_t t0 = 0; t0 < W; t0 += 16384) {
    const uint32_t i0 = t0 + tid * 16;
    uint32_t v[16], tot = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      v[q] = i0 + q < W ? (uint32_t)__popc(crank[i0 + q].x) : 0u;
      tot += v[q];
    }
    const uint32_t x = wave_incl_add(tot);
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    uint32_t base = carry_sh, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
      const uint32_t sw = wsum[w];
      if (w < wid) base += sw;
      all += sw;
    }
    base += x - tot;
    __syncthreads();
    if (tid == 0) carry_sh += all;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      if (i0 + q < W) crank[i0 + q].y = base;
      base += v[q];
    }
    __syncthreads();
  }
  if (tid == 0) {
    crank[W] = make_uint2(0u, carry_sh);
    *n_cols = carry_sh;
  }
}
hipError_t launch_col_rank(const uint64_t *dict_lo, uint32_t C, uint2 *crank, unsigned long long *n_cols,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_crank_bits, dim3((C + 255) / 256), dim3(256), 0, s, dict_lo, C, crank);
  hipLaunchKernelGGL(k_crank_scan, dim3(1), dim3(1024), 0, s, crank, C >> 5, n_cols);
  return hipGetLastError();
}
// per-slot df (the host mirror, vocabulary export, GLOBAL exchange) from the
// per-column df
__global__ void __launch_bounds__(256) k_df_slots(const uint2 *crank, const uint32_t *df_col, uint32_t C,
                                                  uint32_t *df_slot) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= C) return;
  const uint2 e = crank[t >> 5];
  const uint32_t bit = 1u << (t & 31u);
  df_slot[t] = (e.x & bit) ? df_col[e.y + __popc(e.x & (bit - 1u))] : 0u;
}
hipError_t launch_df_slots(const uint2 *crank, const uint32_t *df_col, uint32_t C, uint32_t *df_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_df_slots, dim3((C + 255) / 256), dim3(256), 0, s, crank, df_col, C, df_slot);
  return hipGetLastError();
}

hipError_t launch_block_base(const PostingParams &p, hipStream_t s) {
  hipLaunchKernelGGL(k_block_scan, dim3(1), dim3(1024), 0, s, p);   // (serial k_block_base: 15 us at 123 blocks)
  return hipGetLastError();
}
hipError_t launch_scatter(const PostingParams &p, hipStream_t s) {
  // launch-shape knobs, read per build (A/B and tests/test_gpu_inversion_shapes.py)
  const uint32_t pthreads = [] {
    const char *e = knob("TFIDF_PART_THREADS");
    const int t = e ? atoi(e) : 1024;
    return (uint32_t)(t == 256 || t == 512 ? t : 1024);
  }();
  hipLaunchKernelGGL(k_scatter_part, dim3(tiles_grid(p.n_blocks, p.n_ranges)), dim3(pthreads), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t RS = 1u << p.range_shift;
  const uint32_t nsub = RS > kSubSlots ? RS / kSubSlots : 1u;
  const uint32_t threads = [] {
    const char *e = knob("TFIDF_SORT_THREADS");
    const int t = e ? atoi(e) : 512;                             // 512: 2.89 -> 2.52 ms (cfg 2)
    return (uint32_t)(t == 256 || t == 512 ? t : 1024);
  }();
  hipLaunchKernelGGL(k_scatter_sort, dim3(p.n_blocks, p.n_ranges, (nsub + p.sort_spw - 1) / p.sort_spw), dim3(threads),
                     0, s, p);
  return hipGetLastError();
}

}  // namespace tfidf
