// XCD-partitioned dictionary bound for cfg 5 (round 6).
// The cfg-5 tokenizer probes a 2^23-slot dictionary (64 MB of key words) with
// uniformly random 16 B buckets / 32 B groups; no XCD's 4 MiB L2 holds it, so
// ~94 % of probes are L2 misses served by the Infinity Cache
// (profiles/r05/fetch_calibration.txt).  An XCD-partitioned dictionary would
// let each XCD probe only its own eighth of the key range.  This measures that
// lever's ceiling before building it: the same probes, (a) uniform over the
// whole table, (b) every block confined to the eighth its XCD group owns
// (blockIdx.x % 8 labels the blocks that share an XCD — MI355X_MICROARCH.md),
// (c) the same with the table halved so each eighth fits one L2, and (d) the
// streaming cost of forwarding a probe to its owner and its answer back
// (16 B record out + 4 B answer back, written and read once each, coalesced).
// Times are per launch with HIP events (best of 5 warm launches).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/calib_xcd.hip -o tools/bin/calib_xcd
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

// P probes of W bytes per thread (4 in flight, like the tokenizer's lanes) at
// random W-aligned units of [base, base + n_units) where base is 0 (uniform)
// or the block's XCD group's eighth (parts = 8).
template <int W>
__global__ void __launch_bounds__(256) k_probe(const uint4 *tab, uint64_t n_units, uint32_t parts, uint32_t P,
                                               uint64_t seed, uint32_t *out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t span = n_units / parts;
  const uint64_t base = (uint64_t)(blockIdx.x % parts) * span;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < P; i += 4) {
    uint4 v[4][W / 16];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t u = base + mix(seed ^ (tid * 0x9E3779B97F4A7C15ull) ^ (uint64_t)(i + j)) % span;
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

// Forwarding traffic per probe: write a 16 B record into the owner's queue,
// the owner reads it, writes a 4 B answer, the sender reads the answer —
// modelled as coalesced streams over n records (the queue positions of a real
// design come from a per-XCD atomic cursor; its cost is not modelled here).
__global__ void __launch_bounds__(256) k_forward_out(uint4 *q, uint64_t n, uint64_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix(seed ^ i);
    q[i] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)i, (uint32_t)(i >> 32));
  }
}
__global__ void __launch_bounds__(256) k_forward_answer(const uint4 *q, uint32_t *ans, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 r = q[i];
    ans[i] = r.x ^ r.w;
  }
}
__global__ void __launch_bounds__(256) k_forward_back(const uint32_t *ans, uint64_t n, uint32_t *out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc ^= ans[i];
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t big = 64ull << 20;
  uint4 *tab = nullptr, *q = nullptr;
  uint32_t *out = nullptr, *ans = nullptr;
  const uint32_t blocks = 256 * 8, threads = 256, P = 64;   // 33.5 M probes per launch
  const uint64_t probes = (uint64_t)blocks * threads * P;
  CHECK(hipMalloc(&tab, big));
  CHECK(hipMalloc(&out, (uint64_t)blocks * threads * 4));
  CHECK(hipMalloc(&q, probes * 16));
  CHECK(hipMalloc(&ans, probes * 4));
  CHECK(hipMemset(tab, 1, big));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timed = [&](auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 6; rep++) {                     // rep 0 warms L2 / MALL, not counted
      CHECK(hipEventRecord(e0, 0));
      launch(rep);
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) best = ms < best ? ms : best;
    }
    return best;
  };
  printf("# %llu probes per launch (cfg 5: ~358 M dictionary lookups per tokenizer launch)\n",
         (unsigned long long)probes);
  printf("%-28s %8s %12s\n", "launch", "ms", "G probes/s");
  struct Case { const char *name; int W; uint64_t bytes; uint32_t parts; };
  const Case cases[] = {
      {"probe16_64MiB_uniform", 16, 64ull << 20, 1}, {"probe16_64MiB_xcd8", 16, 64ull << 20, 8},
      {"probe16_32MiB_xcd8", 16, 32ull << 20, 8},    {"probe32_64MiB_uniform", 32, 64ull << 20, 1},
      {"probe32_64MiB_xcd8", 32, 64ull << 20, 8},    {"probe32_32MiB_xcd8", 32, 32ull << 20, 8},
      {"probe16_4MiB_uniform", 16, 4ull << 20, 1},
  };
  for (const Case &c : cases) {
    const uint64_t nu = c.bytes / c.W;
    const float ms = timed([&](int rep) {
      if (c.W == 16)
        hipLaunchKernelGGL(k_probe<16>, dim3(blocks), dim3(threads), 0, 0, tab, nu, c.parts, P, 77 + rep, out);
      else
        hipLaunchKernelGGL(k_probe<32>, dim3(blocks), dim3(threads), 0, 0, tab, nu, c.parts, P, 77 + rep, out);
    });
    printf("%-28s %8.3f %12.1f\n", c.name, ms, probes / (ms * 1e6));
  }
  const uint32_t sblocks = 256 * 8;
  const float f_out = timed([&](int rep) {
    hipLaunchKernelGGL(k_forward_out, dim3(sblocks), dim3(threads), 0, 0, q, probes, (uint64_t)rep);
  });
  const float f_ans = timed([&](int) {
    hipLaunchKernelGGL(k_forward_answer, dim3(sblocks), dim3(threads), 0, 0, q, ans, probes);
  });
  const float f_back = timed([&](int) {
    hipLaunchKernelGGL(k_forward_back, dim3(sblocks), dim3(threads), 0, 0, ans, probes, out);
  });
  printf("%-28s %8.3f %12.1f\n", "forward_record_out_16B", f_out, probes / (f_out * 1e6));
  printf("%-28s %8.3f %12.1f\n", "forward_owner_answer_4B", f_ans, probes / (f_ans * 1e6));
  printf("%-28s %8.3f %12.1f\n", "forward_answer_back", f_back, probes / (f_back * 1e6));
  CHECK(hipFree(tab));
  CHECK(hipFree(out));
  CHECK(hipFree(q));
  CHECK(hipFree(ans));
  return 0;
}
