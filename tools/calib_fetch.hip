// FETCH_SIZE calibration for the tokenizer's dictionary probes (round 5,
// VERDICT r04 item 6).  MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for
// 16 B/lane coalesced streaming reads (it reports half of their bytes), and
// Infinity-Cache (MALL) hits appear to be counted.  The cfg-5 tokenizer reads
// its 2^23-slot dictionary (64 MB of key words) with uniformly random 16 B
// probes (one 2-slot bucket), 32 B probes (4-slot groups) and 128 B windows
// (the retry queue), so its FETCH_SIZE is read here against known byte counts:
// each launch makes a known number of probes of one width into a table of a
// known size (inside L2 / inside the MALL / far beyond it), and rocprofv3
// gives the counters per dispatch (tools/calib_fetch.sh).  Also a coalesced
// 16 B/lane stream as the guide's reference point.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/bin/calib_fetch
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

// Each thread: P probes of W bytes (W / 16 16-B loads, W-aligned) at uniformly
// random positions of a table of n_units W-byte units; probes are independent
// (4 in flight per thread, like the tokenizer's lanes).
template <int W>
__global__ void __launch_bounds__(256) k_probe(const uint4 *tab, uint64_t n_units, uint32_t P, uint64_t seed,
                                               uint32_t *out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < P; i += 4) {
    uint4 v[4][W / 16];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t u = mix(seed ^ (tid * 0x9E3779B97F4A7C15ull) ^ (uint64_t)(i + j)) % n_units;
#pragma unroll
      for (int q = 0; q < W / 16; q++) v[j][q] = tab[u * (W / 16) + q];
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int q = 0; q < W / 16; q++) acc ^= v[j][q].x ^ v[j][q].y ^ v[j][q].z ^ v[j][q].w;
  }
  if (acc == 0x12345678u) out[tid] = acc;   // (keeps the loads; practically never stores)
}

// Coalesced 16 B/lane stream over the first `n` uint4 of the table.
__global__ void __launch_bounds__(256) k_stream(const uint4 *tab, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = tab[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t big = 4ull << 30;                    // 4 GiB table: far beyond the 256 MiB MALL
  uint4 *tab = nullptr;
  uint32_t *out = nullptr;
  CHECK(hipMalloc(&tab, big));
  CHECK(hipMalloc(&out, 64ull << 20));
  CHECK(hipMemset(tab, 1, big));
  const uint32_t blocks = 256 * 8, threads = 256, P = 64;   // 33.5 M probes per launch
  const uint64_t probes = (uint64_t)blocks * threads * P;
  const uint64_t tables[] = {2ull << 20, 64ull << 20, 4ull << 30};   // inside L2, inside the MALL, beyond it
  const char *tnames[] = {"2MiB", "64MiB", "4GiB"};
  printf("dispatch order (one line per launch): name probes bytes_requested\n");
  // stream reference: 1 GiB coalesced
  hipLaunchKernelGGL(k_stream, dim3(blocks), dim3(threads), 0, 0, tab, (1ull << 30) / 16, out);
  CHECK(hipDeviceSynchronize());
  printf("stream16_1GiB %llu %llu\n", (unsigned long long)((1ull << 30) / 16), (unsigned long long)(1ull << 30));
  for (int t = 0; t < 3; t++) {
    for (int w = 0; w < 3; w++) {
      const int W = w == 0 ? 16 : (w == 1 ? 32 : 128);
      // warm the MALL / L2 with one launch first (not counted: the line below names both)
      for (int rep = 0; rep < 2; rep++) {
        const uint64_t nu = tables[t] / W;
        if (W == 16) hipLaunchKernelGGL(k_probe<16>, dim3(blocks), dim3(threads), 0, 0, tab, nu, P, 77 + rep, out);
        else if (W == 32) hipLaunchKernelGGL(k_probe<32>, dim3(blocks), dim3(threads), 0, 0, tab, nu, P, 77 + rep, out);
        else hipLaunchKernelGGL(k_probe<128>, dim3(blocks), dim3(threads), 0, 0, tab, nu, P, 77 + rep, out);
        CHECK(hipDeviceSynchronize());
        printf("probe%d_%s_%s %llu %llu\n", W, tnames[t], rep ? "warm" : "first", (unsigned long long)probes,
               (unsigned long long)(probes * W));
      }
    }
  }
  CHECK(hipFree(tab));
  CHECK(hipFree(out));
  return 0;
}
