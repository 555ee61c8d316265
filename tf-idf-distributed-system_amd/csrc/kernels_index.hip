// kernels_index.hip — index build (Worker.addDocToIndex + IndexWriter.commit
// of the reference, Worker.java:57-94,190-220), hand-written for gfx950.
//
//   tokenize_short : one 256-thread workgroup per document (<= 4 KB).  The
//                    document is staged in LDS by 16 B/lane coalesced loads;
//                    word-break bits are built 64 bytes at a time with a
//                    wavefront ballot (UAX#29 ASCII rules); token spans are
//                    compacted with a block scan; each token is packed into
//                    a 128-bit key and counted in an LDS hash table (the
//                    per-document term histogram = TF); distinct terms are
//                    resolved to dictionary slots in a global open-addressing
//                    table and written as a padded CSR row, grouped by
//                    dictionary range for the DF/inversion passes.
//   tokenize_long  : documents that do not fit the LDS path; chunked, with a
//                    per-document hash table in global memory.
//   df_partial     : per (8192-doc block, 32768-slot range) LDS histogram of
//                    CSR slots -> per-block DF counts (no global atomics).
//   block_scan     : exclusive scan over blocks per slot -> posting offsets,
//                    DF = total (docFreq), in place.
//   col_scan       : exclusive scan of DF -> posting-list start per slot.
//   scatter        : CSR -> block-segmented inverted postings, packed
//                    (doc u32 | tf << 8 | norm) u64.
#include <hip/hip_runtime.h>

#include "tfidf_common.h"
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

__device__ __forceinline__ void set_err(uint32_t *err, uint32_t flag, uint32_t doc) {
  uint32_t old = atomicOr(err, flag);
  if (old == 0) atomicExch(err + 1, doc);
}

// Global dictionary (open addressing, 16 B slots, key lo at [2s], hi at
// [2s+1]).  A lane probes 4 consecutive slots per round with independent
// 16 B loads (one memory round trip covers 4 linear probes).  Claim = CAS on
// the lo word (lo != 0 for every key), then publish hi.  Plain loads may be
// stale but only show an older state (slots go 0 -> key once): a stale
// "empty" falls through to the CAS, which returns the true value.  A slot
// claimed but not yet published is re-read with an agent-scope atomic load.
// SIMT-safe: every claiming lane publishes before any lane re-reads.
__device__ __forceinline__ void probe_pick(ulonglong2 e, uint32_t slot, uint64_t lo, uint64_t hi, uint32_t &js,
                                           int &act) {
  const bool empty = e.x == 0;
  const bool same = e.x == lo && e.y == hi;
  const bool pend = e.x == lo && e.y == 0;
  if (act == 0 && (empty || same || pend)) { js = slot; act = same ? 1 : (empty ? 2 : 3); }
}

__device__ uint32_t dict_find_or_insert(uint64_t *dict, uint32_t mask, uint64_t lo, uint64_t hi, bool active) {
  uint32_t s = key_hash(lo, hi) & mask;
  uint32_t result = kInvalidSlot;
  bool done = !active;
  const uint32_t limit = (mask + 1) + 4096;
  for (uint32_t it = 0; it < limit; it++) {
    if (__all(done)) break;
    uint32_t js = 0;        // slot to act on this round
    int act = 0;            // 0 advance, 1 found, 2 try claim, 3 recheck pending
    if (!done) {
      const uint32_t s1 = (s + 1) & mask, s2 = (s + 2) & mask, s3 = (s + 3) & mask;
      const ulonglong2 e0 = *reinterpret_cast<const ulonglong2 *>(dict + 2 * (size_t)s);
      const ulonglong2 e1 = *reinterpret_cast<const ulonglong2 *>(dict + 2 * (size_t)s1);
      const ulonglong2 e2 = *reinterpret_cast<const ulonglong2 *>(dict + 2 * (size_t)s2);
      const ulonglong2 e3 = *reinterpret_cast<const ulonglong2 *>(dict + 2 * (size_t)s3);
      probe_pick(e0, s, lo, hi, js, act);
      probe_pick(e1, s1, lo, hi, js, act);
      probe_pick(e2, s2, lo, hi, js, act);
      probe_pick(e3, s3, lo, hi, js, act);
      if (act == 0) s = (s + 4) & mask;
      if (act == 1) { result = js; done = true; }
    }
    if (act == 2) {
      unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long *>(dict + 2 * (size_t)js), 0ull,
                                         (unsigned long long)lo);
      if (old == 0) {
        __hip_atomic_store(dict + 2 * (size_t)js + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        result = js;
        done = true;
      } else {
        s = old == lo ? js : ((js + 1) & mask);   // recheck (pending) or move past
      }
    }
    asm volatile("" ::: "memory");
    if (act == 3 && !done) {
      const uint64_t chi = __hip_atomic_load(dict + 2 * (size_t)js + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (chi == hi) { result = js; done = true; }
      else s = chi == 0 ? js : ((js + 1) & mask);
    }
  }
  return result;
}

// Per-document table in global memory (long path).  Only the owning
// workgroup touches it, so workgroup-scope atomics are sufficient.
__device__ uint32_t gtable_insert(uint64_t *keys, uint32_t *cnt, uint32_t mask, uint64_t lo, uint64_t hi) {
  uint32_t s = (key_hash(lo, hi) >> 7) & mask;
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

// Key of the token at LDS buffer bytes [s, e); *valid = false if the span
// holds no letter/digit (only '_' can form such a span).  Tokens of <= 18
// bytes are packed 4 bytes per step: funnel-shift to the token start,
// blank the tail, SWAR lower-case, 4 x 7-bit pack; longer tokens are hashed.
__device__ __forceinline__ uint32_t keep_bytes(uint32_t n, uint32_t i) {   // bytes 4i.. of a token of length n
  return n >= 4 * i + 4 ? 0xFFFFFFFFu : (n <= 4 * i ? 0u : (0xFFFFFFFFu >> (8 * (4 * i + 4 - n))));
}
__device__ __forceinline__ uint32_t pack7(uint32_t t) {
  return (t & 0x7Fu) | (__builtin_amdgcn_ubfe(t, 8, 7) << 7) | (__builtin_amdgcn_ubfe(t, 16, 7) << 14) |
         (__builtin_amdgcn_ubfe(t, 24, 7) << 21);
}
__device__ __forceinline__ uint32_t lower4(uint32_t t) {
  const uint32_t up = (t + 0x3F3F3F3Fu) & ~(t + 0x25252525u) & 0x80808080u;   // 'A'..'Z'
  return t | (up >> 2);
}

__device__ __forceinline__ void token_key(const uint8_t *text, uint32_t s, uint32_t e, uint64_t *lo, uint64_t *hi,
                                          bool *valid) {
  const uint32_t n = e - s;
  if (n > kShortKeyChars) {
    KeyBuilder kb;
    bool any = false;
    for (uint32_t j = s; j < e; j++) {
      const uint8_t c = text[j];
      any |= c != '_';
      kb.push(ascii_lower(c));
    }
    kb.finish(lo, hi);
    *valid = any;
    return;
  }
  const uint32_t *tw = reinterpret_cast<const uint32_t *>(text);
  const uint32_t a0 = s >> 2, o = s & 3;
  const uint32_t d0 = tw[a0], d1 = tw[a0 + 1], d2 = tw[a0 + 2];
  uint32_t t0 = __builtin_amdgcn_alignbyte(d1, d0, o) & keep_bytes(n, 0);
  uint32_t t1 = __builtin_amdgcn_alignbyte(d2, d1, o) & keep_bytes(n, 1);
  uint32_t nu = ((t0 ^ 0x5F5F5F5Fu) & keep_bytes(n, 0)) | ((t1 ^ 0x5F5F5F5Fu) & keep_bytes(n, 1));
  const uint32_t p0 = pack7(lower4(t0)), p1 = pack7(lower4(t1));
  uint32_t p2 = 0, p3 = 0, p4 = 0;
  if (__any(n > 8)) {
    if (n > 8) {
      const uint32_t d3 = tw[a0 + 3], d4 = tw[a0 + 4], d5 = tw[a0 + 5];
      const uint32_t t2 = __builtin_amdgcn_alignbyte(d3, d2, o) & keep_bytes(n, 2);
      const uint32_t t3 = __builtin_amdgcn_alignbyte(d4, d3, o) & keep_bytes(n, 3);
      const uint32_t t4 = __builtin_amdgcn_alignbyte(d5, d4, o) & keep_bytes(n, 4);
      nu |= ((t2 ^ 0x5F5F5F5Fu) & keep_bytes(n, 2)) | ((t3 ^ 0x5F5F5F5Fu) & keep_bytes(n, 3)) |
            ((t4 ^ 0x5F5F5F5Fu) & keep_bytes(n, 4));
      p2 = pack7(lower4(t2));
      p3 = pack7(lower4(t3));
      p4 = pack7(lower4(t4));
    }
  }
  // char j at bit 5 + 7j; group i (4 chars) at bit 5 + 28i; length in bits 0..4
  *lo = (uint64_t)n | ((uint64_t)p0 << 5) | ((uint64_t)p1 << 33) | ((uint64_t)p2 << 61);
  *hi = ((uint64_t)p2 >> 3) | ((uint64_t)p3 << 25) | ((uint64_t)p4 << 53) | kKeyValid;
  *valid = nu != 0;
}

// ---------------------------------------------------------------------------
// Short-document path.

struct ShortSmem {
  uint64_t t_lo[kShortTable];
  uint64_t t_hi[kShortTable];
  uint32_t t_cnt[kShortTable];
  uint16_t claimed[kShortTable];
  uint16_t tok_s[kShortMaxTokens];
  uint16_t tok_e[kShortMaxTokens];
  uint64_t wbits[kShortMaxBytes / 64 + 2];
  uint32_t rcnt[64];
  uint32_t rcur[64];
  uint32_t scan[8];
  uint32_t n_uniq, len, flags, pad;
  uint8_t lut[128];
  alignas(16) uint8_t text[kShortMaxBytes + 64];
};

// Per-document TF histogram in LDS.  One returning ds_cmpst_b64 per probe
// claims an empty slot (lo 0 -> key lo) or reports the resident lo; equal lo
// means equal length, and for tokens of <= 8 bytes equal lo is equality (hi
// is VALID alone), so only longer tokens read hi.  Counting is a
// non-returning ds_add; the list of used slots is built afterwards.
__device__ __forceinline__ void lds_table_insert(ShortSmem &sm, uint64_t lo, uint64_t hi, bool active) {
  uint32_t s = key_hash(lo, hi) >> (32 - 10);           // top 10 bits (kShortTable = 1024)
  const bool short8 = ((uint32_t)(lo & 31) - 1u) < 8u;   // 1..8 bytes (long keys have 0)
  bool done = !active;
  for (uint32_t it = 0; it < kShortTable + 64; it++) {
    if (__all(done)) return;
    uint64_t old = 0;
    if (!done) old = atomicCAS((unsigned long long *)&sm.t_lo[s], 0ull, (unsigned long long)lo);
    const bool claimed = !done && old == 0;
    if (claimed) __hip_atomic_store(&sm.t_hi[s], hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    bool hit = claimed || (!done && old == lo && short8);
    if (!done && !hit && old == lo) {                    // same length > 8: compare hi
      const uint64_t chi = __hip_atomic_load(&sm.t_hi[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (chi == hi) hit = true;
      // chi == 0: claimed by another wave, hi not yet visible -> retry the same slot
      if (chi != hi && chi != 0) s = (s + 1) & (kShortTable - 1);
    } else if (!done && !hit) {
      s = (s + 1) & (kShortTable - 1);
    }
    if (hit) {
      atomicAdd(&sm.t_cnt[s], 1u);
      done = true;
    }
  }
  if (!done) atomicOr(&sm.flags, 2u);   // overflow -> long path
}

// Next-document prefetch into registers: 2 x 16 B per thread covers 4096 +
// 15 bytes of misalignment.  Loads go through an explicit global
// (address_space 1) pointer so they are global_load_dwordx4 and stay in
// flight (nothing waits on them) until the next document is staged.
__device__ __forceinline__ uint4 gload16(const void *ptr) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(1))) const uint32_t gu32;
  gu32 *g = (gu32 *)ptr;
  return make_uint4(g[0], g[1], g[2], g[3]);
#else
  return *reinterpret_cast<const uint4 *>(ptr);
#endif
}

struct DocMeta {
  uint64_t s0, L, src;
  uint32_t shift;
};

__device__ __forceinline__ DocMeta doc_meta(const BuildParams &p, uint64_t d) {
  DocMeta m;
  m.src = p.live_map ? p.live_map[d] : d;
  m.s0 = p.offsets[m.src];
  m.L = p.offsets[m.src + 1] - m.s0;
  m.shift = (uint32_t)(reinterpret_cast<uintptr_t>(p.text + m.s0) & 15);
  return m;
}

__device__ __forceinline__ void prefetch_text(const BuildParams &p, const DocMeta &m, uint4 &v0, uint4 &v1) {
  if (m.L > kShortMaxBytes) return;
  const uint32_t nchunks = (uint32_t)((m.shift + m.L + 15) >> 4);
  const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<uintptr_t>(p.text + m.s0) & ~(uintptr_t)15);
  if (threadIdx.x < nchunks) v0 = gload16(src + threadIdx.x);
  if (threadIdx.x + 256 < nchunks) v1 = gload16(src + threadIdx.x + 256);
}

__global__ void __launch_bounds__(256) k_tokenize_short(BuildParams p) {
  __shared__ ShortSmem sm;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 128; i += 256) sm.lut[i] = wb_class(i);
  for (uint32_t i = tid; i < kShortTable; i += 256) { sm.t_lo[i] = 0; sm.t_hi[i] = 0; sm.t_cnt[i] = 0; }
  if (tid < 64) { sm.rcnt[tid] = 0; sm.rcur[tid] = 0; }
  if (tid == 0) { sm.n_uniq = 0; sm.len = 0; sm.flags = 0; }
  unsigned long long my_doc_count = 0, my_ttf = 0, my_nnz = 0;
  uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
  DocMeta meta;
  if (blockIdx.x < p.n_docs) {
    meta = doc_meta(p, blockIdx.x);
    prefetch_text(p, meta, v0, v1);
  }
  lds_barrier();

  for (uint64_t d = blockIdx.x; d < p.n_docs; d += gridDim.x) {
    const uint64_t src = meta.src, L = meta.L;
    const uint32_t shift = meta.shift;
    const uint64_t dn = d + gridDim.x;
    if (L > kShortMaxBytes) {
      if (tid == 0) p.long_list[atomicAdd(p.long_count, 1u)] = (uint32_t)d;
      if (dn < p.n_docs) { meta = doc_meta(p, dn); prefetch_text(p, meta, v0, v1); }
      continue;                                           // block-uniform
    }
    // stage from registers, then start fetching the next document
    uint4 *dst = reinterpret_cast<uint4 *>(sm.text);
    const uint32_t nchunks = (uint32_t)((shift + L + 15) >> 4);
    if (tid < nchunks) dst[tid] = v0;
    if (tid + 256 < nchunks) dst[tid + 256] = v1;
    if (dn < p.n_docs) { meta = doc_meta(p, dn); prefetch_text(p, meta, v0, v1); }
    lds_barrier();
    if (p.debug_stop == 1) continue;
    const uint32_t lo_b = shift, hi_b = shift + (uint32_t)L;     // document bytes in buffer coordinates
    const bool nonascii = phase_wordbits(sm.text, lo_b, hi_b, sm.wbits, &sm.flags);
    if (nonascii) {
      if (tid == 0) {
        set_err(p.err, kErrNonAscii, (uint32_t)d);
        p.doc_len[d] = 0; p.doc_nuniq[d] = 0; p.doc_norm[d] = 0;
        for (uint32_t r = 0; r < p.n_ranges; r++) p.rsplit[d * p.n_ranges + r] = 0;
        sm.flags = 0;
      }
      lds_barrier();
      continue;
    }
    if (p.debug_stop == 2) continue;
    const uint32_t ntok = phase_token_spans(sm.wbits, hi_b, lo_b, hi_b, sm.tok_s, sm.tok_e, kShortMaxTokens,
                                            sm.scan);
    if (p.debug_stop == 3) continue;
    if (ntok > kShortMaxTokens) {
      if (tid == 0) p.long_list[atomicAdd(p.long_count, 1u)] = (uint32_t)d;
      lds_barrier();
      continue;
    }
    // Phase C: tokens -> per-document histogram in LDS
    uint32_t my_len = 0;
    for (uint32_t i0 = 0; i0 < ntok; i0 += 256) {
      const uint32_t i = i0 + tid;
      uint64_t lo = 0, hi = 0;
      bool valid = false;
      if (i < ntok) {
        const uint32_t s = sm.tok_s[i], e = sm.tok_e[i];
        if (e - s > kMaxTokenLen) {
          set_err(p.err, kErrTokenTooLong, (uint32_t)d);
        } else {
          token_key(sm.text, s, e, &lo, &hi, &valid);
        }
      }
      my_len += valid;
      lds_table_insert(sm, lo, hi, valid);
    }
    atomicAdd(&sm.len, my_len);
    lds_barrier();
    {   // list of used slots: each thread owns 4 consecutive slots
      uint32_t used = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) used |= (sm.t_lo[tid * 4 + q] != 0) << q;
      uint32_t total;
      uint32_t at = block_excl_scan_256(__popc(used), sm.scan, &total);
#pragma unroll
      for (int q = 0; q < 4; q++)
        if (used & (1u << q)) sm.claimed[at++] = (uint16_t)(tid * 4 + q);
      if (tid == 0) sm.n_uniq = total;
      lds_barrier();
    }
    const uint32_t nu = sm.n_uniq;
    if (p.debug_stop == 4) {
      for (uint32_t i = tid; i < nu; i += 256) {
        const uint32_t s = sm.claimed[i];
        sm.t_lo[s] = 0; sm.t_hi[s] = 0; sm.t_cnt[s] = 0;
      }
      lds_barrier();
      if (tid == 0) { sm.n_uniq = 0; sm.len = 0; sm.flags = 0; }
      lds_barrier();
      continue;
    }
    if (sm.flags & 2u) {                                  // LDS table overflow
      for (uint32_t i = tid; i < nu; i += 256) {
        const uint32_t s = sm.claimed[i];
        sm.t_lo[s] = 0; sm.t_hi[s] = 0; sm.t_cnt[s] = 0;
      }
      lds_barrier();
      if (tid == 0) {
        p.long_list[atomicAdd(p.long_count, 1u)] = (uint32_t)d;
        sm.n_uniq = 0; sm.len = 0; sm.flags = 0;
      }
      lds_barrier();
      continue;
    }
    // Phase D: dictionary slots (all lookups of a thread issued together),
    // range partition, CSR row
    const uint64_t base = csr_row_base(p.offsets, src);
    for (uint32_t i0 = 0; i0 < nu; i0 += 256) {
      const uint32_t i = i0 + tid;
      const bool act = i < nu;
      const uint32_t s = act ? sm.claimed[i] : 0;
      uint32_t g = dict_find_or_insert(p.dict, p.cap_mask, act ? sm.t_lo[s] : 1, act ? sm.t_hi[s] : kKeyValid, act);
      if (act) {
        if (g == kInvalidSlot) { set_err(p.err, kErrCapacity, (uint32_t)d); g = 0; }
        atomicAdd(&sm.rcnt[g >> p.range_shift], 1u);
        sm.t_lo[s] = g;
      }
    }
    lds_barrier();
    if (p.debug_stop == 5) {
      for (uint32_t i = tid; i < nu; i += 256) {
        const uint32_t s = sm.claimed[i];
        sm.t_lo[s] = 0; sm.t_hi[s] = 0; sm.t_cnt[s] = 0;
      }
      if (tid < 64) sm.rcnt[tid] = 0;
      lds_barrier();
      if (tid == 0) { sm.n_uniq = 0; sm.len = 0; sm.flags = 0; }
      lds_barrier();
      continue;
    }
    if (tid == 0) {
      uint32_t run = 0;
      for (uint32_t r = 0; r < p.n_ranges; r++) {
        const uint32_t c = sm.rcnt[r];
        sm.rcur[r] = run;
        run += c;
        p.rsplit[d * p.n_ranges + r] = run;
        sm.rcnt[r] = 0;
      }
      const uint32_t len = sm.len;
      p.doc_len[d] = len;
      p.doc_nuniq[d] = nu;
      p.doc_norm[d] = (uint8_t)int_to_byte4(len);
      my_doc_count += len > 0;
      my_ttf += len;
      my_nnz += nu;
    }
    lds_barrier();
    for (uint32_t i = tid; i < nu; i += 256) {
      const uint32_t s = sm.claimed[i];
      const uint32_t g = (uint32_t)sm.t_lo[s];
      const uint32_t pos = atomicAdd(&sm.rcur[g >> p.range_shift], 1u);
      p.csr_col[base + pos] = g;
      p.csr_tf[base + pos] = sm.t_cnt[s];
      sm.t_lo[s] = 0; sm.t_hi[s] = 0; sm.t_cnt[s] = 0;
    }
    lds_barrier();
    if (tid == 0) { sm.n_uniq = 0; sm.len = 0; sm.flags = 0; }
    lds_barrier();
  }
  if (tid == 0) {
    atomicAdd(&p.stats[0], my_doc_count);
    atomicAdd(&p.stats[1], my_ttf);
    atomicAdd(&p.stats[2], my_nnz);
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
    for (uint32_t i = tid; i < T; i += 256) { keys[2 * i] = 0; keys[2 * i + 1] = 0; cnt[i] = 0; }
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
        if (e - s > kMaxTokenLen) { set_err(p.err, kErrTokenTooLong, d); continue; }
        uint64_t lo, hi;
        bool valid;
        token_key(sm.text, s, e, &lo, &hi, &valid);
        if (!valid) continue;
        my_len++;
        if (gtable_insert(keys, cnt, mask, lo, hi) == kInvalidSlot) atomicOr(&sm.flags, 4u);
      }
      __syncthreads();
    }
    if (bad) {
      if (tid == 0) {
        set_err(p.err, kErrNonAscii, d);
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
    for (uint32_t s0 = 0; s0 < T; s0 += 256) {
      const uint32_t s = s0 + tid;
      uint64_t lo = 0, hi = 0;
      if (s < T) {
        lo = __hip_atomic_load(keys + 2 * (size_t)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hi = __hip_atomic_load(keys + 2 * (size_t)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const bool act = lo != 0;
      uint32_t g = dict_find_or_insert(p.dict, p.cap_mask, act ? lo : 1, act ? hi : kKeyValid, act);
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
      p.csr_col[base + pos] = g;
      p.csr_tf[base + pos] = __hip_atomic_load(cnt + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// grid (n_blocks, n_ranges), 1024 threads, LDS histogram of one slot range.
__global__ void __launch_bounds__(1024) k_df_partial(PostingParams p) {
  extern __shared__ uint32_t hist[];
  const uint32_t b = blockIdx.x, r = blockIdx.y;
  const uint32_t RS = 1u << p.range_shift;
  for (uint32_t i = threadIdx.x; i < RS; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const uint64_t d0 = (uint64_t)b * kBlockDocs;
  const uint64_t d1 = d0 + kBlockDocs < p.n_docs ? d0 + kBlockDocs : p.n_docs;
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t rmask = RS - 1;
  for (uint64_t d = d0 + wid; d < d1; d += nw) {
    uint64_t base;
    uint32_t lo, hi;
    doc_segment(p, d, r, &base, &lo, &hi);
    for (uint32_t e = lo + lane; e < hi; e += 64) atomicAdd(&hist[p.csr_col[base + e] & rmask], 1u);
  }
  __syncthreads();
  uint32_t *out = p.blk + (size_t)b * p.C + ((size_t)r << p.range_shift);
  for (uint32_t i = threadIdx.x; i < RS; i += blockDim.x) out[i] = hist[i];
}

// per slot: exclusive scan over blocks in place; row n_blocks = df.
__global__ void __launch_bounds__(256) k_block_scan(PostingParams p) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= p.C) return;
  uint32_t run = 0;
  for (uint32_t b = 0; b < p.n_blocks; b++) {
    const size_t i = (size_t)b * p.C + t;
    const uint32_t v = p.blk[i];
    p.blk[i] = run;
    run += v;
  }
  p.blk[(size_t)p.n_blocks * p.C + t] = run;
}

// single workgroup exclusive scan of df (row n_blocks of blk) -> col_ptr[C + 1].
// Tiles of 16384 slots: each thread loads 16 consecutive df values with four
// 16 B loads (coalesced across the workgroup), scans them in registers, and a
// workgroup scan of the 1024 thread totals gives the offsets.
__global__ void __launch_bounds__(1024) k_col_scan(PostingParams p) {
  __shared__ unsigned long long wsum[16];
  __shared__ unsigned long long carry_sh;
  const uint32_t *df = p.blk + (size_t)p.n_blocks * p.C;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) carry_sh = 0;
  __syncthreads();
  for (uint32_t t0 = 0; t0 < p.C; t0 += 16384) {
    const uint32_t i0 = t0 + tid * 16;
    uint32_t v[16];
    if (i0 + 16 <= p.C) {
      const uint4 *src = reinterpret_cast<const uint4 *>(df + i0);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint4 x = src[q];
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; q++) v[q] = (i0 + q < p.C) ? df[i0 + q] : 0u;
    }
    unsigned long long tot = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) tot += v[q];
    // workgroup exclusive scan of tot
    unsigned long long x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      unsigned long long y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    unsigned long long base = carry_sh, all = 0;
    for (uint32_t w = 0; w < 16; w++) {
      const unsigned long long sw = wsum[w];
      if (w < wid) base += sw;
      all += sw;
    }
    base += x - tot;
    __syncthreads();
    if (tid == 0) carry_sh += all;
    unsigned long long run = base;
    if (i0 < p.C) {
#pragma unroll
      for (int q = 0; q < 16; q++) {
        if (i0 + q < p.C) p.col_ptr[i0 + q] = run;
        run += v[q];
      }
    }
    __syncthreads();
  }
  if (tid == 0) p.col_ptr[p.C] = carry_sh;
}

// grid (n_blocks, n_ranges), 1024 threads: LDS cursor per slot of the range.
__global__ void __launch_bounds__(1024) k_scatter(PostingParams p) {
  extern __shared__ uint32_t cur[];
  const uint32_t b = blockIdx.x, r = blockIdx.y;
  const uint32_t RS = 1u << p.range_shift;
  const size_t g0 = (size_t)r << p.range_shift;
  for (uint32_t i = threadIdx.x; i < RS; i += blockDim.x)
    cur[i] = (uint32_t)(p.col_ptr[g0 + i] + p.blk[(size_t)b * p.C + g0 + i]);
  __syncthreads();
  const uint64_t d0 = (uint64_t)b * kBlockDocs;
  const uint64_t d1 = d0 + kBlockDocs < p.n_docs ? d0 + kBlockDocs : p.n_docs;
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t rmask = RS - 1;
  for (uint64_t d = d0 + wid; d < d1; d += nw) {
    uint64_t base;
    uint32_t lo, hi;
    doc_segment(p, d, r, &base, &lo, &hi);
    const uint32_t nrm = p.doc_norm[d];
    for (uint32_t e = lo + lane; e < hi; e += 64) {
      const uint32_t g = p.csr_col[base + e];
      const uint32_t tf = p.csr_tf[base + e];
      if (tf > kMaxTf) atomicOr(p.err, kErrTfTooLarge);
      const uint32_t pos = atomicAdd(&cur[g & rmask], 1u);
      p.post[pos] = (uint64_t)(uint32_t)d | ((uint64_t)((tf << 8) | nrm) << 32);
    }
  }
}

// ---------------------------------------------------------------------------
// launchers

hipError_t launch_tokenize_short(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_short, dim3(grid), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_tokenize_long(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_long, dim3(grid), dim3(256), 0, s, p);
  return hipGetLastError();
}
static void allow_big_lds() {
  static bool done = false;
  if (done) return;
  hipFuncSetAttribute((const void *)k_df_partial, hipFuncAttributeMaxDynamicSharedMemorySize, 4 << kRangeBits);
  hipFuncSetAttribute((const void *)k_scatter, hipFuncAttributeMaxDynamicSharedMemorySize, 4 << kRangeBits);
  done = true;
}

hipError_t launch_df_partial(const PostingParams &p, hipStream_t s) {
  allow_big_lds();
  const size_t lds = sizeof(uint32_t) << p.range_shift;
  hipLaunchKernelGGL(k_df_partial, dim3(p.n_blocks, p.n_ranges), dim3(1024), lds, s, p);
  return hipGetLastError();
}
hipError_t launch_block_scan(const PostingParams &p, hipStream_t s) {
  hipLaunchKernelGGL(k_block_scan, dim3((p.C + 255) / 256), dim3(256), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_col_scan(const PostingParams &p, hipStream_t s) {
  hipLaunchKernelGGL(k_col_scan, dim3(1), dim3(1024), 0, s, p);
  return hipGetLastError();
}
hipError_t launch_scatter(const PostingParams &p, hipStream_t s) {
  allow_big_lds();
  const size_t lds = sizeof(uint32_t) << p.range_shift;
  hipLaunchKernelGGL(k_scatter, dim3(p.n_blocks, p.n_ranges), dim3(1024), lds, s, p);
  return hipGetLastError();
}

}  // namespace tfidf
