// wave_ops.h — wave-level helpers shared by the index and query kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tfidf {

// Lanes of the wave holding the same BITS-bit key (active lanes only): one
// ballot per key bit.  Used to turn same-address LDS atomics (hot terms hit
// one cursor from most lanes of a wave) into one atomic per distinct key.
template <int BITS>
__device__ __forceinline__ uint64_t peer_mask(uint32_t key) {
  uint64_t peers = __ballot(1);
#pragma unroll
  for (int b = 0; b < BITS; b++) {
    const uint64_t m = __ballot((key >> b) & 1u);
    peers &= ((key >> b) & 1u) ? m : ~m;
  }
  return peers;
}

// Wave-aggregated cursor bump: returns the old cursor value + this lane's rank
// among its peers (same result as one atomicAdd(cur + key, 1) per lane).
template <int BITS>
__device__ __forceinline__ uint32_t cursor_bump(uint32_t *cur, uint32_t key, uint32_t lane) {
  const uint64_t peers = peer_mask<BITS>(key);
  const uint32_t rank = (uint32_t)__popcll(peers & ((1ull << lane) - 1));
  const uint32_t leader = (uint32_t)__builtin_ctzll(peers);
  uint32_t base = 0;
  if (rank == 0) base = atomicAdd(cur + key, (uint32_t)__popcll(peers));
  base = (uint32_t)__shfl((int)base, (int)leader, 64);
  return base + rank;
}

}  // namespace tfidf
