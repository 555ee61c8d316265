// kernels_synth.hip — synthetic Zipf corpus generator (bench/test input,
// SURVEY.md §8(d)) + small utility kernels.  Must match
// tfidf_amd/synth.py bit for bit (tests/test_synth.py checks it).
//
//   mix64 = splitmix64 step (tfidf_common.h); S2 = mix64(seed)
//   doc d (global id), T_d = len_min + mix64(S2 ^ (d << 20 | 0xFFFFF)) % (len_max - len_min + 1)
//   token t:  u = (mix64(S2 ^ (d << 20 | t)) >> 11) * 2^-53
//             rank = 1 + #{i : cdf[i] <= u}           (searchsorted right)
//   word(rank) = bijective base-26 of (rank + 18278), 'a' = 1
//   separator after token t: '\n' if t % 16 == 15 or t == T_d - 1, else ' '
#include <hip/hip_runtime.h>

#include "tfidf_common.h"
#include "tfidf_internal.h"

namespace tfidf {

constexpr uint32_t kGuideBits = 16;

__device__ __forceinline__ uint32_t synth_rank(uint64_t h, const double *cdf, const uint32_t *guide, uint32_t V) {
  const double u = (double)(h >> 11) * 0x1.0p-53;
  const uint32_t g = (uint32_t)(u * (double)(1u << kGuideBits));
  uint32_t lo = guide[g], hi = guide[g + 1];       // answer index in [lo, hi]
  while (lo < hi) {                                 // first i with cdf[i] > u
    const uint32_t mid = (lo + hi) >> 1;
    if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
  }
  return lo + 1 <= V ? lo + 1 : V;
}

__device__ __forceinline__ uint32_t word_len(uint32_t rank) {
  uint64_t n = (uint64_t)rank + 18278ull;
  uint32_t len = 0;
  while (n) { n = (n - 1) / 26; len++; }
  return len;
}

__device__ __forceinline__ uint32_t doc_tokens(uint64_t s2, uint64_t d, uint32_t len_min, uint32_t len_max) {
  const uint64_t h = mix64(s2 ^ ((d << 20) | 0xFFFFFull));
  return len_min + (uint32_t)(h % (uint64_t)(len_max - len_min + 1));
}

// one wave per document
__global__ void __launch_bounds__(256) k_synth_lengths(uint64_t seed, uint64_t n_docs, uint64_t doc_base,
                                                       const double *cdf, const uint32_t *guide, uint32_t V,
                                                       uint32_t len_min, uint32_t len_max, uint64_t *bytes) {
  const uint64_t s2 = mix64(seed);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t i = w; i < n_docs; i += nw) {
    const uint64_t d = doc_base + i;
    const uint32_t T = doc_tokens(s2, d, len_min, len_max);
    uint64_t sum = 0;
    for (uint32_t t = lane; t < T; t += 64)
      sum += word_len(synth_rank(mix64(s2 ^ ((d << 20) | t)), cdf, guide, V)) + 1;
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_down(sum, o, 64);
    if (lane == 0) bytes[i] = sum;
  }
}

__global__ void __launch_bounds__(256) k_synth_text(uint64_t seed, uint64_t n_docs, uint64_t doc_base,
                                                    const double *cdf, const uint32_t *guide, uint32_t V,
                                                    uint32_t len_min, uint32_t len_max, const uint64_t *offsets,
                                                    uint8_t *text) {
  const uint64_t s2 = mix64(seed);
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t i = w; i < n_docs; i += nw) {
    const uint64_t d = doc_base + i;
    const uint32_t T = doc_tokens(s2, d, len_min, len_max);
    uint64_t pos = offsets[i];
    for (uint32_t t0 = 0; t0 < T; t0 += 64) {
      const uint32_t t = t0 + lane;
      uint32_t rank = 0, len = 0;
      if (t < T) {
        rank = synth_rank(mix64(s2 ^ ((d << 20) | t)), cdf, guide, V);
        len = word_len(rank);
      }
      // wave inclusive scan of (len + 1)
      uint32_t x = t < T ? len + 1 : 0, incl = x;
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += y;
      }
      if (t < T) {
        uint8_t *out = text + pos + (incl - x);
        uint64_t n = (uint64_t)rank + 18278ull;
        for (int j = (int)len - 1; j >= 0; j--) {
          n -= 1;
          out[j] = (uint8_t)('a' + (n % 26));
          n /= 26;
        }
        out[len] = (t % 16 == 15 || t == T - 1) ? '\n' : ' ';
      }
      pos += __shfl(incl, 63, 64);
    }
  }
}

// single-workgroup exclusive scan (n up to ~1e9; bandwidth of one CU is
// ample for corpus setup, which is outside every timed region).
__global__ void __launch_bounds__(1024) k_excl_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n) {
  __shared__ unsigned long long part[1024];
  const uint64_t per = (n + 1023) / 1024;
  const uint64_t a = (uint64_t)threadIdx.x * per;
  const uint64_t z = a + per < n ? a + per : n;
  unsigned long long s = 0;
  for (uint64_t i = a; i < z; i++) s += in[i];
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
    const uint64_t v = in[i];
    out[i] = run;
    run += v;
  }
  if (threadIdx.x == 1023) out[n] = part[1023];
}

hipError_t synth_doc_lengths(uint64_t seed, uint64_t n_docs, uint64_t doc_base, const double *cdf,
                             const uint32_t *guide, uint32_t V, uint32_t len_min, uint32_t len_max,
                             uint64_t *bytes_out, hipStream_t s) {
  const uint64_t blocks = (n_docs * 64 + 255) / 256;
  const int grid = (int)(blocks < 8192 ? (blocks ? blocks : 1) : 8192);
  hipLaunchKernelGGL(k_synth_lengths, dim3(grid), dim3(256), 0, s, seed, n_docs, doc_base, cdf, guide, V, len_min,
                     len_max, bytes_out);
  return hipGetLastError();
}

hipError_t synth_doc_text(uint64_t seed, uint64_t n_docs, uint64_t doc_base, const double *cdf,
                          const uint32_t *guide, uint32_t V, uint32_t len_min, uint32_t len_max,
                          const uint64_t *offsets, uint8_t *text, hipStream_t s) {
  const uint64_t blocks = (n_docs * 64 + 255) / 256;
  const int grid = (int)(blocks < 8192 ? (blocks ? blocks : 1) : 8192);
  hipLaunchKernelGGL(k_synth_text, dim3(grid), dim3(256), 0, s, seed, n_docs, doc_base, cdf, guide, V, len_min,
                     len_max, offsets, text);
  return hipGetLastError();
}

hipError_t exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_excl_scan_u64, dim3(1), dim3(1024), 0, s, in, out, n);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// vocabulary helpers for GLOBAL statistics

__global__ void k_add_u64(uint64_t *v, uint64_t n, uint64_t delta) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] += delta;
}

hipError_t add_u64(uint64_t *v, uint64_t n, uint64_t delta, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_add_u64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, v, n, delta);
  return hipGetLastError();
}

// canonical keys (sorted by (hi, lo)) are searched for each local slot key
__global__ void k_slot_to_canon(const uint64_t *dict, uint32_t C, const uint64_t *canon, uint64_t n_canon,
                                uint32_t *canon_of_slot) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= C) return;
  const uint64_t lo = dict[s], hi = dict[C + s];   // lo[C] then hi[C]
  if (lo == 0) { canon_of_slot[s] = kInvalidSlot; return; }
  uint64_t a = 0, z = n_canon;
  while (a < z) {
    const uint64_t m = (a + z) >> 1;
    const uint64_t mh = canon[2 * m + 1], ml = canon[2 * m];
    if (mh < hi || (mh == hi && ml < lo)) a = m + 1; else z = m;
  }
  canon_of_slot[s] = (a < n_canon && canon[2 * a] == lo && canon[2 * a + 1] == hi) ? (uint32_t)a : kInvalidSlot;
}

__global__ void k_scatter_df_canon(const uint32_t *df, const uint32_t *canon_of_slot, uint32_t C, uint32_t *out) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= C) return;
  const uint32_t c = canon_of_slot[s];
  if (c != kInvalidSlot) out[c] = df[s];
}

__global__ void k_gather_df_canon(const uint32_t *dfc, const uint32_t *canon_of_slot, uint32_t C, uint32_t *gdf) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= C) return;
  const uint32_t c = canon_of_slot[s];
  gdf[s] = c != kInvalidSlot ? dfc[c] : 0u;
}

hipError_t slot_to_canon(const uint64_t *dict, uint32_t C, const uint64_t *canon, uint64_t n_canon,
                         uint32_t *canon_of_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_slot_to_canon, dim3((C + 255) / 256), dim3(256), 0, s, dict, C, canon, n_canon, canon_of_slot);
  return hipGetLastError();
}
hipError_t scatter_df_canon(const uint32_t *df, const uint32_t *canon_of_slot, uint32_t C, uint32_t *out,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_scatter_df_canon, dim3((C + 255) / 256), dim3(256), 0, s, df, canon_of_slot, C, out);
  return hipGetLastError();
}
hipError_t gather_df_canon(const uint32_t *dfc, const uint32_t *canon_of_slot, uint32_t C, uint32_t *gdf,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_gather_df_canon, dim3((C + 255) / 256), dim3(256), 0, s, dfc, canon_of_slot, C, gdf);
  return hipGetLastError();
}

}  // namespace tfidf
