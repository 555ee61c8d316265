// kernels_sort.hip — device sorts built on rocPRIM/hipCUB radix sort (tools
// and tests only; the all-hits order is kernels_query.hip's merge passes):
//   * canonical vocabulary for GLOBAL statistics: sorted union of 128-bit
//     term keys, ordered by (hi, lo), de-duplicated.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "tfidf_common.h"
#include "tfidf_internal.h"

namespace tfidf {

hipError_t exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s);

__global__ void k_split128(const uint64_t *keys, uint64_t n, uint64_t *lo, uint64_t *hi, uint32_t *idx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  lo[i] = keys[2 * i];
  hi[i] = keys[2 * i + 1];
  idx[i] = (uint32_t)i;
}

__global__ void k_gather_u64(const uint64_t *src, const uint32_t *idx, uint64_t n, uint64_t *dst) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

// flags[i] = 1 if key i starts a run (and is a valid key: hi != 0)
__global__ void k_unique_flags(const uint64_t *lo_sorted_src, const uint32_t *idx, const uint64_t *hi_sorted,
                               uint64_t n, uint64_t *flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t h = hi_sorted[i], l = lo_sorted_src[idx[i]];
  bool start = h != 0;
  if (i > 0 && start) start = !(hi_sorted[i - 1] == h && lo_sorted_src[idx[i - 1]] == l);
  flags[i] = start ? 1 : 0;
}

__global__ void k_unique_write(const uint64_t *lo_src, const uint32_t *idx, const uint64_t *hi_sorted,
                               const uint64_t *flags, const uint64_t *pos, uint64_t n, uint64_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !flags[i]) return;
  const uint64_t p = pos[i];
  out[2 * p] = lo_src[idx[i]];
  out[2 * p + 1] = hi_sorted[i];
}

// keys: n x (lo, hi); out: unique sorted keys; *n_unique written (host).
// Keys with hi == 0 (padding) are dropped.
hipError_t sort_unique_keys128(const uint64_t *keys, uint64_t n, uint64_t *out, uint64_t *n_unique, hipStream_t s) {
  *n_unique = 0;
  if (n == 0) return hipSuccess;
  hipError_t e;
  uint64_t *lo = nullptr, *hi = nullptr, *lo_s = nullptr, *hi_g = nullptr, *hi_s = nullptr, *flags = nullptr,
           *pos = nullptr;
  uint32_t *idx = nullptr, *idx1 = nullptr, *idx2 = nullptr;
  void *tmp = nullptr;
  size_t tmp_bytes = 0, t2 = 0;
  const unsigned g = (unsigned)((n + 255) / 256);
#define TRY(x) do { e = (x); if (e != hipSuccess) goto done; } while (0)
  TRY(hipMallocAsync((void **)&lo, n * 8, s));
  TRY(hipMallocAsync((void **)&hi, n * 8, s));
  TRY(hipMallocAsync((void **)&lo_s, n * 8, s));
  TRY(hipMallocAsync((void **)&hi_g, n * 8, s));
  TRY(hipMallocAsync((void **)&hi_s, n * 8, s));
  TRY(hipMallocAsync((void **)&flags, n * 8, s));
  TRY(hipMallocAsync((void **)&pos, (n + 1) * 8, s));
  TRY(hipMallocAsync((void **)&idx, n * 4, s));
  TRY(hipMallocAsync((void **)&idx1, n * 4, s));
  TRY(hipMallocAsync((void **)&idx2, n * 4, s));
  hipLaunchKernelGGL(k_split128, dim3(g), dim3(256), 0, s, keys, n, lo, hi, idx);
  TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, lo, lo_s, idx, idx1, (int)n, 0, 64, s));
  TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, t2, hi, hi_s, idx, idx2, (int)n, 0, 64, s));
  if (t2 > tmp_bytes) tmp_bytes = t2;
  TRY(hipMallocAsync(&tmp, tmp_bytes, s));
  // LSD: by lo, then stable by hi
  TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, lo, lo_s, idx, idx1, (int)n, 0, 64, s));
  hipLaunchKernelGGL(k_gather_u64, dim3(g), dim3(256), 0, s, hi, idx1, n, hi_g);
  TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, hi_g, hi_s, idx1, idx2, (int)n, 0, 64, s));
  hipLaunchKernelGGL(k_unique_flags, dim3(g), dim3(256), 0, s, lo, idx2, hi_s, n, flags);
  TRY(exclusive_scan_u64(flags, pos, n, s));
  hipLaunchKernelGGL(k_unique_write, dim3(g), dim3(256), 0, s, lo, idx2, hi_s, flags, pos, n, out);
  TRY(hipMemcpyAsync(n_unique, pos + n, 8, hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
done:
#undef TRY
  hipFreeAsync(lo, s); hipFreeAsync(hi, s); hipFreeAsync(lo_s, s); hipFreeAsync(hi_g, s);
  hipFreeAsync(hi_s, s); hipFreeAsync(flags, s); hipFreeAsync(pos, s);
  hipFreeAsync(idx, s); hipFreeAsync(idx1, s); hipFreeAsync(idx2, s); hipFreeAsync(tmp, s);
  return e;
}

}  // namespace tfidf
