// dict_device.h — the global term dictionary's device-side find-or-insert,
// shared by the index build (kernels_index.hip) and the distributed
// vocabulary reduction (kernels_vocab.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tfidf_common.h"

namespace tfidf {

// Global dictionary: lo[C], hi[C], ref[C] (u64 each).  ref holds one
// occurrence of a hashed key's term (dict_ref_word: text offset and byte
// length), written by the claimer, read by the exact-identity checks.  Probing is linear
// over the slots starting at the aligned 2-slot bucket of key_hash & (C - 1);
// one 16 B load of lo covers a bucket.  Claim = CAS lo 0 -> key lo, then
// publish hi (agent scope).  A resident lo equal to the lo of a key of <= 8
// bytes IS that key (lo holds every byte; bit 63 clear), so such keys never
// read hi; other keys compare hi, re-reading a claimed-but-unpublished hi (0).
// Slots go 0 -> key once, so a stale plain load only shows an older state: a
// stale "empty" falls through to the CAS, which returns the true value.
__device__ __forceinline__ bool key_lo_is_short(uint64_t lo) { return (lo >> 63) == 0; }

// reference occurrence word: bit 63 | byte length << 40 | text offset
TFIDF_HD uint64_t dict_ref_word(uint64_t off, uint32_t len) { return (1ull << 63) | ((uint64_t)len << 40) | off; }
TFIDF_HD uint64_t dict_ref_off(uint64_t r) { return r & ((1ull << 40) - 1); }
TFIDF_HD uint32_t dict_ref_len(uint64_t r) { return (uint32_t)(r >> 40) & 0x3FFu; }

// ref (optional): per key, the reference word a successful claim of a hashed
// key stores; claimed (optional): whether this lane claimed the slot.
template <int K>
__device__ __forceinline__ void dict_lookup_multi(uint64_t *dict, uint32_t mask, const uint64_t *lo, const uint64_t *hi,
                                                  const bool *act, uint32_t *out, const uint64_t *ref = nullptr,
                                                  bool *claimed = nullptr) {
  uint64_t *dlo = dict;
  uint64_t *dhi = dict + (size_t)mask + 1;
  if (claimed)
#pragma unroll
    for (int j = 0; j < K; j++) claimed[j] = false;
  uint32_t s[K];
  bool done[K];
#pragma unroll
  for (int j = 0; j < K; j++) {
    s[j] = dict_home(dict_hash(lo[j], hi[j]), mask) & ~1u;
    done[j] = !act[j];
    out[j] = kInvalidSlot;
  }
  const uint32_t limit = mask + 1 + 4096;
  for (uint32_t it = 0; it < limit; it++) {
    bool anyp = false;
#pragma unroll
    for (int j = 0; j < K; j++) anyp |= !done[j];
    if (!__any(anyp)) break;
    ulonglong2 e[K];
#pragma unroll
    for (int j = 0; j < K; j++)
      if (!done[j]) e[j] = *reinterpret_cast<const ulonglong2 *>(dlo + (s[j] & ~1u));
    uint32_t js[K];
    int a[K];     // 0 advance, 1 found, 2 try claim, 3 compare hi
#pragma unroll
    for (int j = 0; j < K; j++) {
      a[j] = 0;
      js[j] = s[j];
      if (!done[j]) {
        const bool sh = key_lo_is_short(lo[j]);
        const uint64_t v0 = (s[j] & 1) ? e[j].y : e[j].x;
        if (v0 == 0) a[j] = 2;
        else if (v0 == lo[j]) a[j] = sh ? 1 : 3;
        else if (!(s[j] & 1)) {
          js[j] = s[j] + 1;
          if (e[j].y == 0) a[j] = 2;
          else if (e[j].y == lo[j]) a[j] = sh ? 1 : 3;
        }
        if (a[j] == 0) s[j] = ((s[j] | 1u) + 1u) & mask;
        if (a[j] == 1) { out[j] = js[j]; done[j] = true; }
      }
    }
#pragma unroll
    for (int j = 0; j < K; j++) {
      if (a[j] == 2) {
        const unsigned long long old =
            atomicCAS(reinterpret_cast<unsigned long long *>(dlo + js[j]), 0ull, (unsigned long long)lo[j]);
        if (old == 0) {
          if (ref && (lo[j] & kLoHashed))
            __hip_atomic_store(dict + 2 * ((size_t)mask + 1) + js[j], ref[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(dhi + js[j], hi[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          out[j] = js[j];
          done[j] = true;
          if (claimed) claimed[j] = true;
        } else if (old == lo[j]) {
          if (key_lo_is_short(lo[j])) { out[j] = js[j]; done[j] = true; }
          else { s[j] = js[j]; a[j] = 3; }
        } else {
          s[j] = (js[j] + 1) & mask;
        }
      }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < K; j++) {
      if (a[j] == 3 && !done[j]) {
        const uint64_t chi = __hip_atomic_load(dhi + js[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (chi == hi[j]) { out[j] = js[j]; done[j] = true; }
        else s[j] = chi == 0 ? js[j] : ((js[j] + 1) & mask);
      }
    }
  }
}

__device__ __forceinline__ uint32_t dict_find_or_insert(uint64_t *dict, uint32_t mask, uint64_t lo, uint64_t hi,
                                                        bool active, const uint64_t *ref = nullptr,
                                                        bool *claimed = nullptr) {
  uint32_t out;
  dict_lookup_multi<1>(dict, mask, &lo, &hi, &active, &out, ref, claimed);
  return out;
}

}  // namespace tfidf
