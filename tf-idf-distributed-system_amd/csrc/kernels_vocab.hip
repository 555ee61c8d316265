// kernels_vocab.hip — GLOBAL statistics by term ownership.
//
// The reference's single worker sees one docFreq per term (Lucene
// CollectionStatistics/TermStatistics at J/worker/Worker.java:230).  With the
// corpus sharded over G GPUs every shard counts its own docFreq; the global
// value is the sum over shards of the same term.  Each term has an owner rank
// (hash of its 128-bit key mod G):
//   1. partition : every shard groups its (key, df) records by owner;
//   2. all-to-all (RCCL, host orchestration) sends each group to its owner;
//   3. reduce    : the owner sums df over identical keys in a device hash table
//                  (the dictionary's own find-or-insert) and answers, record by
//                  record, with the summed df;
//   4. all-to-all back, then each shard scatters the answers into a per-slot
//      global-df vector.
// Work per rank is O(vocabulary / G x G) = O(vocabulary), independent of G, and
// nothing is sorted.
#include <hip/hip_runtime.h>

#include "dict_device.h"
#include "tfidf_common.h"
#include "tfidf_internal.h"

namespace tfidf {

__device__ __forceinline__ uint32_t owner_of(uint64_t lo, uint64_t hi, uint32_t G) {
  uint32_t x = dict_hash(lo, hi) * 0x85EBCA6Bu;     // bits independent of the dictionary's home slot
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return (uint32_t)(((uint64_t)x * G) >> 32);
}

// Per-owner counts / record positions: a workgroup histograms its slots'
// owners in LDS and takes one global atomic per (workgroup, owner) — the
// global counters are G addresses, so per-record global atomics serialise
// (cfg 2, 100 k terms, G = 1: 2.3 ms for the two passes).
constexpr uint32_t kVocabThreads = 256;
constexpr uint32_t kVocabMaxG = 1024;

__global__ void __launch_bounds__(kVocabThreads) k_vocab_count(const uint64_t *dict, uint32_t C, uint32_t G,
                                                                uint32_t *counts) {
  __shared__ uint32_t c[kVocabMaxG];
  for (uint32_t r = threadIdx.x; r < G; r += blockDim.x) c[r] = 0;
  __syncthreads();
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = s < C ? dict[s] : 0;
  if (lo != 0) atomicAdd(&c[owner_of(lo, dict[(size_t)C + s], G)], 1u);
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < G; r += blockDim.x)
    if (c[r]) atomicAdd(&counts[r], c[r]);
}

__global__ void __launch_bounds__(kVocabThreads) k_vocab_scatter(const uint64_t *dict, const uint32_t *df, uint32_t C,
                                                                  uint32_t G, uint32_t *cursor, uint64_t *records,
                                                                  uint32_t *sent_slot) {
  __shared__ uint32_t c[kVocabMaxG];
  for (uint32_t r = threadIdx.x; r < G; r += blockDim.x) c[r] = 0;
  __syncthreads();
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = s < C ? dict[s] : 0;
  uint64_t hi = 0;
  uint32_t own = 0, rank = 0;
  if (lo != 0) {
    hi = dict[(size_t)C + s];
    own = owner_of(lo, hi, G);
    rank = atomicAdd(&c[own], 1u);
  }
  __syncthreads();
  for (uint32_t r = threadIdx.x; r < G; r += blockDim.x)
    if (c[r]) c[r] = atomicAdd(&cursor[r], c[r]);            // this workgroup's range of owner r
  __syncthreads();
  if (lo != 0) {
    const uint32_t at = c[own] + rank;
    records[3 * (size_t)at] = lo;
    records[3 * (size_t)at + 1] = hi;
    records[3 * (size_t)at + 2] = df[s];
    sent_slot[at] = s;
  }
}

// (distinct terms: the claims, counted here — round 5 scanned the whole owner
// table afterwards, 51 us of the one-rank exchange)
__global__ void k_vocab_insert(const uint64_t *records, uint64_t n, uint64_t *table, uint32_t tmask, uint32_t *sums,
                               uint32_t *rslot, unsigned long long *n_unique) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = i < n;
  const uint64_t lo = act ? records[3 * i] : 1, hi = act ? records[3 * i + 1] : kKeyValid;
  bool cl = false;
  const uint32_t slot = dict_find_or_insert(table, tmask, lo, hi, act, nullptr, &cl);
  if (act) {
    atomicAdd(&sums[slot], (uint32_t)records[3 * i + 2]);
    rslot[i] = slot;
  }
  const uint64_t m = __ballot(act && cl);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(n_unique, (unsigned long long)__popcll(m));
}

__global__ void k_vocab_answer(const uint32_t *sums, const uint32_t *rslot, uint64_t n, uint32_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = sums[rslot[i]];
}

__global__ void k_vocab_import(const uint32_t *sent_slot, const uint32_t *gdf_in, uint64_t n, uint32_t *gdf) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) gdf[sent_slot[i]] = gdf_in[i];
}

// per-owner record counts -> exclusive start cursors (u32) and the caller's
// u64 counts; G <= 1024, one workgroup
__global__ void k_vocab_starts(const uint32_t *counts, uint32_t G, uint32_t *cursor, uint64_t *counts_out) {
  __shared__ uint32_t c[1024];
  for (uint32_t r = threadIdx.x; r < G; r += blockDim.x) c[r] = counts[r];
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t r = 0; r < G; r++) { cursor[r] = acc; acc += c[r]; }
  }
  for (uint32_t r = threadIdx.x; r < G; r += blockDim.x) counts_out[r] = c[r];
}

static unsigned blocks(uint64_t n) { return (unsigned)((n + 255) / 256 ? (n + 255) / 256 : 1); }

hipError_t vocab_count(const uint64_t *dict, uint32_t C, uint32_t G, uint32_t *counts, hipStream_t s) {
  if (G > kVocabMaxG) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_vocab_count, dim3(blocks(C)), dim3(kVocabThreads), 0, s, dict, C, G, counts);
  return hipGetLastError();
}

hipError_t vocab_starts(const uint32_t *counts, uint32_t G, uint32_t *cursor, uint64_t *counts_out, hipStream_t s) {
  hipLaunchKernelGGL(k_vocab_starts, dim3(1), dim3(256), 0, s, counts, G, cursor, counts_out);
  return hipGetLastError();
}

hipError_t vocab_scatter(const uint64_t *dict, const uint32_t *df, uint32_t C, uint32_t G, uint32_t *cursor,
                         uint64_t *records, uint32_t *sent_slot, hipStream_t s) {
  if (G > kVocabMaxG) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_vocab_scatter, dim3(blocks(C)), dim3(kVocabThreads), 0, s, dict, df, C, G, cursor, records,
                     sent_slot);
  return hipGetLastError();
}

hipError_t vocab_reduce(const uint64_t *records, uint64_t n, uint64_t *table, uint32_t tmask, uint32_t *sums,
                        uint32_t *rslot, uint32_t *out, unsigned long long *n_unique, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_vocab_insert, dim3(blocks(n)), dim3(256), 0, s, records, n, table, tmask, sums, rslot, n_unique);
  hipLaunchKernelGGL(k_vocab_answer, dim3(blocks(n)), dim3(256), 0, s, sums, rslot, n, out);
  return hipGetLastError();
}

hipError_t vocab_import(const uint32_t *sent_slot, const uint32_t *gdf_in, uint64_t n, uint32_t *gdf, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_vocab_import, dim3(blocks(n)), dim3(256), 0, s, sent_slot, gdf_in, n, gdf);
  return hipGetLastError();
}

}  // namespace tfidf
