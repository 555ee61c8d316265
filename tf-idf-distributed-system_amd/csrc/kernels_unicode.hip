// kernels_unicode.hip — index build of documents holding non-ASCII text
// (Worker.addDocToIndex, Worker.java:190-220, through StandardAnalyzer's full
// Unicode grammar; unicode_scan.h), hand-written for gfx950.
//
//   tokenize_uwave : one wavefront per document (aligned window <= 4 KB), the
//                    documents the ASCII wave path found a byte >= 0x80 in.
//                    The document is staged in LDS; lane l scans the slice
//                    [cut_l, cut_{l+1}) with the longest-match DFA, cuts just
//                    after ASCII class-OTHER bytes (the scanner's start state
//                    holds there); every round each lane yields at most one
//                    token, keyed (lower-cased UTF-8 -> 128-bit key), and the
//                    wave inserts the round's keys into a 1024-slot LDS table
//                    (64-bit CAS on lo, then hi; in-order LDS within the wave
//                    makes the winner's hi visible to the losers of the same
//                    round).  Distinct terms are resolved in the global
//                    dictionary (8 lookups per lane in flight) and written as
//                    a CSR row grouped by dictionary range, as the other
//                    tokenizer paths do.  Documents that do not fit (window,
//                    > 768 distinct terms, malformed UTF-8) go to the long path.
#include <hip/hip_runtime.h>

#include "dict_device.h"
#include "tfidf_common.h"
#include "tfidf_internal.h"
#include "unicode_scan.h"

namespace tfidf {

constexpr uint32_t kUwWindow = 4096;
constexpr uint32_t kUwSlots = 1024;
constexpr uint32_t kUwSlotBits = 10;
constexpr uint32_t kUwMaxTerms = 768;
constexpr uint32_t kUwMaxRanges = 64;

struct UwSmem {
  alignas(16) uint8_t text[kUwWindow + 16];
  unsigned long long klo[kUwSlots];   // key lo; after the lookup: dictionary slot
  unsigned long long khi[kUwSlots];   // key hi (VALID bit set: occupied)
  uint32_t cnt[kUwSlots];             // tf
  uint32_t rcnt[kUwMaxRanges];        // per-range counts, then cursors
};

__device__ __forceinline__ uint32_t uw_incl_add(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  return x;
}

__global__ void __launch_bounds__(64) k_tokenize_uwave(BuildParams p) {
  __shared__ UwSmem sm;
  const uint32_t lane = threadIdx.x;
  const uint32_t n_uni = *p.uni_count;
  const uint32_t R = p.n_ranges;
  unsigned long long my_dc = 0, my_ttf = 0, my_nnz = 0;

  for (uint32_t it = blockIdx.x; it < n_uni; it += gridDim.x) {
    const uint32_t d = p.uni_list[it];
    const uint64_t src = p.live_map ? p.live_map[d] : d;
    const uint64_t s0 = p.offsets[src];
    const uint64_t L = p.offsets[src + 1] - s0;
    if (L > kUwWindow || R > kUwMaxRanges) {                // wave-uniform
      if (lane == 0) p.long_list[atomicAdd(p.long_count, 1u)] = d;
      continue;
    }
    // ---- stage (aligned 16 B loads) + clear the table
    const uintptr_t a = reinterpret_cast<uintptr_t>(p.text + s0);
    const uint32_t shift = (uint32_t)(a & 15);
    const uint32_t nchunks = (uint32_t)((shift + L + 15) >> 4);
    const uint4 *gsrc = reinterpret_cast<const uint4 *>(a - shift);
    uint4 *dst = reinterpret_cast<uint4 *>(sm.text);
    for (uint32_t c = lane; c < nchunks; c += 64) dst[c] = gsrc[c];
    for (uint32_t s = lane; s < kUwSlots; s += 64) { sm.klo[s] = 0; sm.khi[s] = 0; sm.cnt[s] = 0; }
    sm.rcnt[lane] = 0;
    __syncthreads();
    const uint8_t *doc = sm.text + shift;

    // ---- slices: lane l scans tokens starting in [cut(l), cut(l + 1))
    const uint64_t seg = (L + 63) >> 6;
    auto cut = [&](uint64_t t) -> uint64_t {
      if (t == 0) return 0;
      uint64_t q = t * seg;
      if (q >= L) return L;
      while (q < L && !uc_split_byte(doc[q - 1])) q++;
      return q;
    };
    uint64_t pos = cut(lane);
    const uint64_t stop = cut(lane + 1);
    bool active = pos < stop, ubad = false, overflow = false;
    uint32_t ntok = 0;
    while (__any(active)) {
      uint64_t ts, te, lo = 0, hi = 0;
      bool have = false;
      if (active) {
        have = uc_next_token(doc, L, &pos, stop, &ts, &te, &lo, &hi, &ubad);
        active = have;
      }
      ntok += have;
      // round insert: probe from the key's home slot, linear
      uint32_t slot = dict_hash(lo, hi) >> (32 - kUwSlotBits);
      bool done = !have;
      for (uint32_t r = 0; r < kUwSlots && __any(!done); r++) {
        unsigned long long old = 1;
        if (!done) old = atomicCAS(&sm.klo[slot], 0ull, (unsigned long long)lo);
        const bool won = !done && old == 0;
        if (won) sm.khi[slot] = hi;
        asm volatile("" ::: "memory");
        bool match = false;
        if (!done && !won && old == lo) match = sm.khi[slot] == hi;
        if (won || match) {
          atomicAdd(&sm.cnt[slot], 1u);
          done = true;
        } else if (!done) {
          slot = (slot + 1) & (kUwSlots - 1);
        }
      }
      overflow |= !done;
    }
    // ---- distinct terms; documents the wave cannot take go to the long path
    uint32_t occ = 0;
    for (uint32_t s = lane; s < kUwSlots; s += 64) occ += sm.khi[s] != 0;
    const uint32_t nu = (uint32_t)__builtin_amdgcn_readlane((int)uw_incl_add(occ, lane), 63);
    if (__any(ubad) || __any(overflow) || nu > kUwMaxTerms) {   // wave-uniform
      if (lane == 0) p.long_list[atomicAdd(p.long_count, 1u)] = d;
      __syncthreads();
      continue;
    }
    const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)uw_incl_add(ntok, lane), 63);
    // ---- dictionary slots (8 lookups per lane in flight), range counts
#pragma unroll
    for (int h = 0; h < 2; h++) {
      uint64_t klo[8], khi[8];
      bool act[8];
      uint32_t g[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t s = lane + 64 * (8 * h + k);
        klo[k] = sm.klo[s];
        khi[k] = sm.khi[s];
        act[k] = khi[k] != 0;
        if (!act[k]) { klo[k] = 1; khi[k] = kKeyValid; }
      }
      dict_lookup_multi<8>(p.dict, p.cap_mask, klo, khi, act, g);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (!act[k]) continue;
        uint32_t gs = g[k];
        if (gs == kInvalidSlot) { atomicOr(p.err, kErrCapacity); gs = 0; }
        sm.klo[lane + 64 * (8 * h + k)] = gs;
        atomicAdd(&sm.rcnt[gs >> p.range_shift], 1u);
      }
    }
    __syncthreads();
    // ---- row segments: inclusive ends per range, cursors = exclusive starts
    {
      const uint32_t c = lane < R ? sm.rcnt[lane] : 0u;
      const uint32_t incl = uw_incl_add(c, lane);
      if (lane < R) {
        p.rsplit[(uint64_t)d * R + lane] = incl;
        sm.rcnt[lane] = incl - c;
      }
    }
    __syncthreads();
    const uint64_t base = csr_row_base(p.offsets, src);
    for (uint32_t s = lane; s < kUwSlots; s += 64) {
      if (sm.khi[s] == 0) continue;
      const uint32_t gs = (uint32_t)sm.klo[s];
      const uint32_t at = atomicAdd(&sm.rcnt[gs >> p.range_shift], 1u);
      p.csr_col[base + at] = gs;
      p.csr_tf[base + at] = sm.cnt[s];
    }
    if (lane == 0) {
      p.doc_len[d] = len;
      p.doc_nuniq[d] = nu;
      p.doc_norm[d] = (uint8_t)int_to_byte4(len);
      my_dc += len > 0;
      my_ttf += len;
      my_nnz += nu;
    }
    __syncthreads();
  }
  if (lane == 0 && (my_ttf | my_nnz)) {
    atomicAdd(&p.stats[0], my_dc);
    atomicAdd(&p.stats[1], my_ttf);
    atomicAdd(&p.stats[2], my_nnz);
  }
}

hipError_t launch_tokenize_uwave(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_uwave, dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace tfidf
