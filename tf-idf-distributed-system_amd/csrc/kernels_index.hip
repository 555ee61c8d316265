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
__device__ uint32_t dict_find_or_insert(uint64_t *dict, uint32_t mask, uint64_t lo, uint64_t hi, bool active) {
  uint32_t s = (uint32_t)key_hash(lo, hi) & mask;
  uint32_t result = kInvalidSlot;
  bool done = !active;
  const uint32_t limit = (mask + 1) + 4096;
  for (uint32_t it = 0; it < limit; it++) {
    if (__all(done)) break;
    uint32_t js = 0;        // slot to act on this round
    int act = 0;            // 0 advance, 1 found, 2 try claim, 3 recheck pending
    if (!done) {
      ulonglong2 e[4];
#pragma unroll
      for (int j = 0; j < 4; j++) e[j] = *reinterpret_cast<const ulonglong2 *>(dict + 2 * (size_t)((s + j) & mask));
#pragma unroll
      for (int j = 3; j >= 0; j--) {   // earliest slot wins
        const bool empty = e[j].x == 0;
        const bool same = e[j].x == lo && e[j].y == hi;
        const bool pend = e[j].x == lo && e[j].y == 0;
        if (empty || same || pend) { js = (s + j) & mask; act = same ? 1 : (empty ? 2 : 3); }
      }
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
  uint32_t s = (uint32_t)key_hash(lo, hi) & mask;
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

__device__ __forceinline__ uint8_t code_at(const uint8_t *text, const uint8_t *lut, uint32_t shift, int64_t r,
                                           int64_t wlen) {
  if (r < 0 || r >= wlen) return 0;
  uint8_t c = text[shift + r];
  return lut[c & 127];
}

// Word-segment bits, 64 positions per wave-iteration: one LDS byte read +
// one class-LUT read per lane; neighbour classes by lane shuffle (only lanes
// 0 and 63 read across the 64-byte boundary); the membership bits of the
// 64 positions are one __ballot.  Returns true (block-uniform) if a
// non-ASCII byte is present.
__device__ bool phase_wordbits(const uint8_t *text, const uint8_t *lut, uint32_t shift, uint32_t wlen,
                               uint64_t *wbits, uint32_t *flag_lds) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t nwords = (wlen + 63) >> 6;
  bool nonascii = false;
  for (uint32_t m = wid; m < nwords; m += 4) {
    const int64_t r = (int64_t)m * 64 + lane;
    uint32_t cur = 0;
    if (r < wlen) {
      const uint8_t c = text[shift + r];
      nonascii |= c >= 128;
      cur = lut[c & 127];
    }
    uint32_t prev = __shfl_up(cur, 1, 64);
    uint32_t next = __shfl_down(cur, 1, 64);
    if (lane == 0) prev = code_at(text, lut, shift, r - 1, wlen);
    if (lane == 63) next = code_at(text, lut, shift, r + 1, wlen);
    const bool w = (r < wlen) && wb_is_word((uint8_t)prev, (uint8_t)cur, (uint8_t)next);
    const uint64_t mask = __ballot(w);
    if (lane == 0) wbits[m] = mask;
  }
  if (__any(nonascii) && lane == 0) atomicOr(flag_lds, 1u);
  lds_barrier();
  const bool bad = (*flag_lds & 1u) != 0;
  lds_barrier();      // every thread has read the flag before anyone resets it
  return bad;
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

// Key of the token [s, e) of the window; *valid = false if the span holds no
// letter/digit (a run of '_' is not a token).  The 7-bit packing is exact
// for <= 18 bytes; only longer tokens pay for the two hashes.
__device__ __forceinline__ void token_key(const uint8_t *text, const uint8_t *lut, uint32_t shift, uint32_t s,
                                          uint32_t e, uint64_t *lo, uint64_t *hi, bool *valid) {
  const uint32_t n = e - s;
  uint8_t any = 0;
  if (n <= kShortKeyChars) {
    uint64_t a = 0, b = 0;
    for (uint32_t j = 0; j < n; j++) {
      const uint8_t c = text[shift + s + j];
      any |= lut[c & 127];
      const uint64_t v = ascii_lower(c);
      const uint32_t bit = 7 * j;
      if (bit < 64) a |= v << bit;
      if (bit + 7 > 64) b |= bit < 64 ? (v >> (64 - bit)) : (v << (bit - 64));
    }
    *lo = a;
    *hi = b | kKeyValid;
  } else {
    KeyBuilder kb;
    for (uint32_t j = s; j < e; j++) {
      const uint8_t c = text[shift + j];
      any |= lut[c & 127];
      kb.push(ascii_lower(c));
    }
    kb.finish(lo, hi);
  }
  *valid = (any & (kClsL | kClsD)) != 0;
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

__device__ __forceinline__ void lds_table_insert(ShortSmem &sm, uint64_t lo, uint64_t hi, bool active) {
  uint32_t s = (uint32_t)key_hash(lo, hi) & (kShortTable - 1);
  bool done = !active;
  for (uint32_t it = 0; it < 2 * kShortTable + 256; it++) {
    if (__all(done)) return;
    bool claimed = false;
    uint64_t clo = 0, chi = 0;
    if (!done) {
      clo = *(volatile uint64_t *)&sm.t_lo[s];
      if (clo == 0) {
        unsigned long long old = atomicCAS((unsigned long long *)&sm.t_lo[s], 0ull, (unsigned long long)lo);
        if (old == 0) {
          *(volatile uint64_t *)&sm.t_hi[s] = hi;
          atomicAdd(&sm.t_cnt[s], 1u);
          const uint32_t idx = atomicAdd(&sm.n_uniq, 1u);
          sm.claimed[idx] = (uint16_t)s;
          claimed = true;
          done = true;
        } else {
          clo = old;
        }
      }
    }
    asm volatile("" ::: "memory");
    if (!done && !claimed) {
      if (clo == lo) {
        chi = *(volatile uint64_t *)&sm.t_hi[s];
        if (chi == hi) {
          atomicAdd(&sm.t_cnt[s], 1u);
          done = true;
        } else if (chi != 0) {
          s = (s + 1) & (kShortTable - 1);
        }
        // chi == 0: claimed by another wave, not yet published -> retry slot
      } else {
        s = (s + 1) & (kShortTable - 1);
      }
    }
  }
  if (!done) atomicOr(&sm.flags, 2u);   // overflow -> long path
}

// Prefetch of a short document's bytes into registers: 2 x 16 B per thread
// covers 4096 + 15 bytes of misalignment.
struct DocPrefetch {
  uint4 v0, v1;
  uint64_t s0, L, src;
  uint32_t shift;
  bool valid;
};

__device__ __forceinline__ void prefetch_doc(const BuildParams &p, uint64_t d, DocPrefetch &pf) {
  pf.valid = d < p.n_docs;
  if (!pf.valid) return;
  pf.src = p.live_map ? p.live_map[d] : d;
  pf.s0 = p.offsets[pf.src];
  pf.L = p.offsets[pf.src + 1] - pf.s0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p.text + pf.s0);
  const uintptr_t al = a & ~(uintptr_t)15;
  pf.shift = (uint32_t)(a - al);
  if (pf.L > kShortMaxBytes) return;
  const uint32_t nchunks = (uint32_t)((pf.shift + pf.L + 15) >> 4);
  const uint4 *src = reinterpret_cast<const uint4 *>(al);
  const uint4 z = make_uint4(0, 0, 0, 0);
  pf.v0 = threadIdx.x < nchunks ? src[threadIdx.x] : z;
  pf.v1 = threadIdx.x + 256 < nchunks ? src[threadIdx.x + 256] : z;
}

__global__ void __launch_bounds__(256) k_tokenize_short(BuildParams p) {
  __shared__ ShortSmem sm;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 128; i += 256) sm.lut[i] = wb_class(i);
  for (uint32_t i = tid; i < kShortTable; i += 256) { sm.t_lo[i] = 0; sm.t_hi[i] = 0; sm.t_cnt[i] = 0; }
  if (tid < 64) { sm.rcnt[tid] = 0; sm.rcur[tid] = 0; }
  if (tid == 0) { sm.n_uniq = 0; sm.len = 0; sm.flags = 0; }
  unsigned long long my_doc_count = 0, my_ttf = 0, my_nnz = 0;
  DocPrefetch pf;
  prefetch_doc(p, blockIdx.x, pf);
  lds_barrier();

  for (uint64_t d = blockIdx.x; d < p.n_docs; d += gridDim.x) {
    const uint64_t src = pf.src, L = pf.L;
    const uint32_t shift = pf.shift;
    if (L > kShortMaxBytes) {
      if (tid == 0) p.long_list[atomicAdd(p.long_count, 1u)] = (uint32_t)d;
      prefetch_doc(p, d + gridDim.x, pf);
      continue;                                           // block-uniform
    }
    // stage from registers, then start fetching the next document
    uint4 *dst = reinterpret_cast<uint4 *>(sm.text);
    const uint32_t nchunks = (uint32_t)((shift + L + 15) >> 4);
    if (tid < nchunks) dst[tid] = pf.v0;
    if (tid + 256 < nchunks) dst[tid + 256] = pf.v1;
    prefetch_doc(p, d + gridDim.x, pf);
    lds_barrier();
    const bool nonascii = phase_wordbits(sm.text, sm.lut, shift, (uint32_t)L, sm.wbits, &sm.flags);
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
    const uint32_t ntok = phase_token_spans(sm.wbits, (uint32_t)L, 0, (uint32_t)L, sm.tok_s, sm.tok_e,
                                            kShortMaxTokens, sm.scan);
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
          token_key(sm.text, sm.lut, shift, s, e, &lo, &hi, &valid);
        }
      }
      my_len += valid;
      lds_table_insert(sm, lo, hi, valid);
    }
    atomicAdd(&sm.len, my_len);
    lds_barrier();
    const uint32_t nu = sm.n_uniq;
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
      if (phase_wordbits(sm.text, sm.lut, shift, wlen, sm.wbits, &sm.flags)) { bad = true; break; }
      const uint32_t ntok = phase_token_spans(sm.wbits, wlen, (uint32_t)(cs - wlo), (uint32_t)(ce - wlo),
                                              sm.tok_s, sm.tok_e, kChunk / 2 + 8, sm.scan);
      for (uint32_t i = tid; i < ntok; i += 256) {
        const uint32_t s = sm.tok_s[i], e = sm.tok_e[i];
        if (e - s > kMaxTokenLen) { set_err(p.err, kErrTokenTooLong, d); continue; }
        uint64_t lo, hi;
        bool valid;
        token_key(sm.text, sm.lut, shift, s, e, &lo, &hi, &valid);
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

// single workgroup exclusive scan of df (row n_blocks of blk) -> col_ptr[C + 1]
__global__ void __launch_bounds__(1024) k_col_scan(PostingParams p) {
  __shared__ unsigned long long part[1024];
  const uint32_t *df = p.blk + (size_t)p.n_blocks * p.C;
  const uint32_t per = (p.C + 1023) / 1024;
  const uint64_t a = (uint64_t)threadIdx.x * per;
  const uint64_t z = a + per < p.C ? a + per : p.C;
  unsigned long long s = 0;
  for (uint64_t i = a; i < z; i++) s += df[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    unsigned long long v = threadIdx.x >= o ? part[threadIdx.x - o] : 0ull;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  unsigned long long run = part[threadIdx.x] - s;
  for (uint64_t i = a; i < z; i++) {
    p.col_ptr[i] = run;
    run += df[i];
  }
  if (threadIdx.x == 1023) p.col_ptr[p.C] = part[1023];
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
