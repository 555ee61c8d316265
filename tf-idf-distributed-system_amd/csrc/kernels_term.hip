// kernels_term.hip — term-major inversion for large vocabularies.
//
// The block-major inversion (kernels_index.hip) keeps a dense per-block count
// table of (N / 8192 + 1) x C words.  With SURVEY §8 cfg 5 (5 M-term vocabulary,
// millions of short documents per GPU) that table alone would be tens of GB, so
// above a size threshold the index is inverted term-major instead: postings
// sorted by (term, doc).  The input rows are already in document order, so the
// inversion is a STABLE sort of the (doc, term) entries by term.  Hand-written
// here as an LSD radix sort over one packed 64-bit word per entry:
//
//   key = slot | doc | min(tf, esc) | norm, fields from the top: log2 C slot
//         bits, ceil(log2 N) doc bits, the rest less 8 for tf, the norm byte
//         (cfg-5 shape: 23 | 23 | 10 | 8; at most 26 | 26 | 4 | 8)
//
//   1. row offsets: exclusive scan of the documents' distinct-term counts;
//   2. k_term_pairs: one wave per document writes its row's packed words at
//      its row offset (document order); a tf the field cannot hold goes to an
//      escape list of (slot << 26 | doc, tf) pairs;
//   3. per 8-bit digit of the slot bits, low digit first:
//        k_rs_hist    per tile of 8192 words, the digit histogram (LDS),
//                     stored digit-major: hist[digit][tile];
//        scan         exclusive scan of hist -> each (digit, tile) run's
//                     output start (digit-major order = stable order);
//        k_rs_scatter per tile: stable rank of every word among the tile's
//                     words of its digit (each wave ranks a quarter of the
//                     tile in input order against its own digit counters;
//                     per-wave bases by one scan), words placed in LDS in digit order, then
//                     written out digit run by digit run (coalesced); the
//                     LAST pass writes the postings doc | (tf << 8 | norm)
//                     << 32 instead, and adds each (tile, term) run's length
//                     to df[term] (two atomics per run);
//   4. toff = exclusive scan of df.
//
// Bytes per posting: 12 (pairs) + 3 passes x (8 hist + 16 scatter) for
// 2^17..2^24-slot dictionaries (rocPRIM's pair sort: 12 B key + value words
// per pass, plus pairs, copy and bounds: ~100 B).
//
// The result is what Lucene's postings hold for the field (per term, docs in
// ascending order with freq and the doc's norm byte) — reference: inversion
// inside IndexWriter.updateDocument, J/worker/Worker.java:218; read back by
// searcher.search at :230.
#include <hip/hip_runtime.h>

#include "tfidf_common.h"
#include "tfidf_internal.h"
#include "wave_ops.h"

namespace tfidf {

constexpr uint32_t kTermDocBits = 26;                   // escape-list key: slot << 26 | doc
#ifndef TFIDF_RS_THREADS
#define TFIDF_RS_THREADS 512
#endif
constexpr uint32_t kRsThreads = TFIDF_RS_THREADS;      // radix tile = kRsThreads x kRsItems words (>= 256 threads;
                                                        // 8192-word tiles: digit runs twice as long, cfg-5 sort
                                                        // 8.08 -> 7.61 ms; 16384 (one workgroup per CU) 9.34)
constexpr uint32_t kRsItems = 16;                       // words per thread per tile
constexpr uint32_t kRsTile = kRsThreads * kRsItems;     // 8192
constexpr uint32_t kRsWaves = kRsThreads / 64;

// ---------------------------------------------------------------------------
// exclusive scan of u32 (n <= 2^32 - 1 total): per-block sums, one-block scan
// of the block sums, then the block-local scans plus bases.
constexpr uint32_t kScanThreads = 1024, kScanItems = 16, kScanBlock = kScanThreads * kScanItems;

__device__ __forceinline__ uint32_t block_incl_scan(uint32_t x, uint32_t *wsum, uint32_t *total) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (uint32_t w = 0; w < nw; w++) {
    const uint32_t v = wsum[w];
    if (w < wid) base += v;
    all += v;
  }
  __syncthreads();
  *total = all;
  return base + x;
}

__global__ void __launch_bounds__(kScanThreads) k_scan_sums(const uint32_t *in, uint64_t n, uint32_t *sums) {
  __shared__ uint32_t wsum[16];
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock;
  uint32_t s = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; j++) {
    const uint64_t i = b0 + (uint64_t)j * kScanThreads + threadIdx.x;
    s += i < n ? in[i] : 0u;
  }
  uint32_t tot;
  block_incl_scan(s, wsum, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// one workgroup: exclusive scan of nb block sums in place (nb <= 2^20)
__global__ void __launch_bounds__(kScanThreads) k_scan_top(uint32_t *sums, uint32_t nb) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint32_t c0 = 0; c0 < nb; c0 += kScanThreads) {
    const uint32_t i = c0 + threadIdx.x;
    const uint32_t v = i < nb ? sums[i] : 0u;
    uint32_t tot;
    const uint32_t incl = block_incl_scan(v, wsum, &tot);
    const uint32_t base = carry;
    if (i < nb) sums[i] = base + incl - v;
    __syncthreads();
    if (threadIdx.x == 0) carry = base + tot;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kScanThreads) k_scan_final(const uint32_t *in, uint64_t n, const uint32_t *sums,
                                                             uint32_t *out) {
  __shared__ uint32_t wsum[16];
  const uint64_t b0 = (uint64_t)blockIdx.x * kScanBlock;
  // thread t scans its kScanItems consecutive words (one strided pass of the
  // block's words per item index keeps the loads coalesced)
  uint32_t v[kScanItems], s = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; j++) {
    const uint64_t i = b0 + (uint64_t)threadIdx.x * kScanItems + j;
    v[j] = i < n ? in[i] : 0u;
    s += v[j];
  }
  uint32_t tot;
  uint32_t run = sums[blockIdx.x] + block_incl_scan(s, wsum, &tot) - s;
#pragma unroll
  for (uint32_t j = 0; j < kScanItems; j++) {
    const uint64_t i = b0 + (uint64_t)threadIdx.x * kScanItems + j;
    if (i < n) out[i] = run;
    run += v[j];
  }
}

// scratch: ceil(n / kScanBlock) words
static hipError_t scan_u32_excl(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *scratch, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
  hipLaunchKernelGGL(k_scan_sums, dim3(nb), dim3(kScanThreads), 0, s, in, n, scratch);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanThreads), 0, s, scratch, nb);
  hipLaunchKernelGGL(k_scan_final, dim3(nb), dim3(kScanThreads), 0, s, in, n, scratch, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Packed word fields (TermParams.doc_bits / tf_bits, slot_bits = log2 C)
struct TermLayout {
  uint32_t sb, db, tb;                 // slot, doc, tf bits; norm = 8
  __host__ __device__ uint32_t slot_shift() const { return 64 - sb; }
  __host__ __device__ uint32_t doc_shift() const { return 8 + tb; }
  __host__ __device__ uint32_t tf_esc() const { return (1u << tb) - 1; }
  __host__ __device__ uint64_t pack(uint32_t slot, uint64_t doc, uint32_t tf, uint32_t norm) const {
    return ((uint64_t)slot << slot_shift()) | (doc << doc_shift()) | ((uint64_t)(tf < tf_esc() ? tf : tf_esc()) << 8) |
           norm;
  }
};

// Four documents per wave (16 lanes each, grid-stride): the rows are
// contiguous, so each lane group writes consecutive words; the four rows'
// metadata loads are in flight together (short rows: ~57 words at cfg 5).
__global__ void __launch_bounds__(256) k_term_pairs(TermParams p) {
  const uint32_t lane = threadIdx.x & 63, grp = lane >> 4, sl = lane & 15;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t esc = csr_esc_value(p.slot_bits);
  const TermLayout ly{p.slot_bits, p.doc_bits, p.tf_bits};
  for (uint64_t d0 = 4 * wave; d0 < p.n_docs; d0 += 4 * nw) {
    const uint64_t d = d0 + grp;
    if (d >= p.n_docs) continue;
    const uint64_t src = p.live_map ? p.live_map[d] : d;
    const uint64_t base = csr_row_base(p.offsets, src);
    const uint32_t n = p.doc_nuniq[d], o = p.row_off[d], nrm = p.doc_norm[d];
    for (uint32_t j = sl; j < n; j += 16) {
      const uint32_t e = p.csr[base + j], c = csr_local(e, p.slot_bits);
      uint32_t t = csr_tf_field(e, p.slot_bits);
      if (t == esc) t = csr_esc_tf(p.csr_esc, p.n_esc, base + j);
      if (t > kMaxTf) atomicOr(p.err, kErrTfTooLarge);
      if (t >= ly.tf_esc()) {                                  // rare: exact tf kept aside, keyed (slot, doc)
        const uint32_t at = atomicAdd(p.tesc_count, 1u);
        if (at < p.tesc_cap) {                                 // (slot << 26 | doc, tf) pairs
          p.tesc[2 * (uint64_t)at] = ((uint64_t)c << kTermDocBits) | d;
          p.tesc[2 * (uint64_t)at + 1] = min(t, kMaxTf);
        }
      }
      p.keys[o + j] = ly.pack(c, d, t, nrm);
    }
  }
}

// Long rows (book-sized documents, SURVEY cfg 1: ~24 k distinct terms per
// row, a few hundred rows): four documents per wave would leave most of the
// chip idle (300 books -> 75 waves), so workgroup (x, y) takes entries
// y * 256 + t, stepping by gridDim.y * 256, of documents x, x + gridDim.x, ...
__global__ void __launch_bounds__(256) k_term_pairs_wide(TermParams p) {
  const uint32_t esc = csr_esc_value(p.slot_bits);
  const TermLayout ly{p.slot_bits, p.doc_bits, p.tf_bits};
  for (uint64_t d = blockIdx.x; d < p.n_docs; d += gridDim.x) {
    const uint64_t src = p.live_map ? p.live_map[d] : d;
    const uint64_t base = csr_row_base(p.offsets, src);
    const uint32_t n = p.doc_nuniq[d], o = p.row_off[d], nrm = p.doc_norm[d];
    for (uint32_t j = blockIdx.y * blockDim.x + threadIdx.x; j < n; j += gridDim.y * blockDim.x) {
      const uint32_t e = p.csr[base + j], c = csr_local(e, p.slot_bits);
      uint32_t t = csr_tf_field(e, p.slot_bits);
      if (t == esc) t = csr_esc_tf(p.csr_esc, p.n_esc, base + j);
      if (t > kMaxTf) atomicOr(p.err, kErrTfTooLarge);
      if (t >= ly.tf_esc()) {
        const uint32_t at = atomicAdd(p.tesc_count, 1u);
        if (at < p.tesc_cap) {
          p.tesc[2 * (uint64_t)at] = ((uint64_t)c << kTermDocBits) | d;
          p.tesc[2 * (uint64_t)at + 1] = min(t, kMaxTf);
        }
      }
      p.keys[o + j] = ly.pack(c, d, t, nrm);
    }
  }
}

// Tile-aligned form (round 3): workgroup t writes exactly the words of radix
// tile t (indices [t, t + 1) * kRsTile, starting inside document tile_doc[t])
// and stores the tile's histogram of the first radix digit (the slot's low
// bits), so the sort's first k_rs_hist pass — a full read of the words — is
// not needed.  Each wave walks four documents per step (16 lanes each) on its
// own, until its documents start past the tile; a document that straddles a
// tile boundary is split between the two workgroups.
__global__ void __launch_bounds__(256) k_term_pairs_tiled(TermParams p, const uint32_t *tile_doc, uint32_t *hist) {
  __shared__ uint32_t h[256];
  const uint32_t tid = threadIdx.x, lane = tid & 63, grp = lane >> 4, sl = lane & 15, wid = tid >> 6;
  h[tid] = 0;
  __syncthreads();
  const uint32_t esc = csr_esc_value(p.slot_bits);
  const TermLayout ly{p.slot_bits, p.doc_bits, p.tf_bits};
  const uint32_t mask0 = (1u << (p.slot_bits < 8 ? p.slot_bits : 8)) - 1;
  const uint64_t i0 = (uint64_t)blockIdx.x * kRsTile, i1 = min(i0 + kRsTile, p.nnz);
  for (uint64_t db = tile_doc[blockIdx.x];; db += 16) {
    const uint64_t d = db + 4 * wid + grp;
    bool before_end = false;
    if (d < p.n_docs) {
      const uint64_t o = p.row_off[d];
      before_end = o < i1;
      if (before_end) {
        const uint32_t n = p.doc_nuniq[d];
        const uint64_t jlo = o < i0 ? i0 - o : 0, jhi = min((uint64_t)n, i1 - o);
        if (jlo < jhi) {
          const uint64_t src = p.live_map ? p.live_map[d] : d;
          const uint64_t base = csr_row_base(p.offsets, src);
          const uint32_t nrm = p.doc_norm[d];
          for (uint64_t j = jlo + sl; j < jhi; j += 16) {
            const uint32_t e = p.csr[base + j], c = csr_local(e, p.slot_bits);
            uint32_t t = csr_tf_field(e, p.slot_bits);
            if (t == esc) t = csr_esc_tf(p.csr_esc, p.n_esc, base + j);
            if (t > kMaxTf) atomicOr(p.err, kErrTfTooLarge);
            if (t >= ly.tf_esc()) {                                // rare: exact tf kept aside, keyed (slot, doc)
              const uint32_t at = atomicAdd(p.tesc_count, 1u);
              if (at < p.tesc_cap) {
                p.tesc[2 * (uint64_t)at] = ((uint64_t)c << kTermDocBits) | d;
                p.tesc[2 * (uint64_t)at + 1] = min(t, kMaxTf);
              }
            }
            p.keys[o + j] = ly.pack(c, d, t, nrm);
            atomicAdd(&h[c & mask0], 1u);
          }
        }
      }
    }
    if (!__any(before_end)) break;                             // documents are in row order (wave-uniform)
  }
  __syncthreads();
  hist[(uint64_t)blockIdx.x * 256 + tid] = h[tid];
}

// tile t's first word lies in the row of document tile_doc[t]
__global__ void k_tile_docs(const uint32_t *row_off, const uint32_t *nuniq, uint64_t n_docs, uint32_t *tile_doc) {
  const uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_docs) return;
  const uint64_t o = row_off[d], n = nuniq[d];
  for (uint64_t t = (o + kRsTile - 1) / kRsTile; t * kRsTile < o + n; t++) tile_doc[t] = (uint32_t)d;
}

// ---------------------------------------------------------------------------
// LSD radix passes (8-bit digits of the key bits from `shift`)

__device__ __forceinline__ uint32_t rs_digit(uint64_t k, uint32_t shift, uint32_t mask) {
  return (uint32_t)(k >> shift) & mask;
}

// per tile: digit histogram -> hist[tile * 256 + digit] (tile-major: one
// coalesced 1 KB row per tile; the digit-major [digit][tile] layout of round
// 2 stored 256 scattered words per tile — 0.82 GB of HBM writes for an 85 MB
// table at cfg 5 — and the scatter pass read it back with the same stride)
__global__ void __launch_bounds__(kRsThreads) k_rs_hist(const uint64_t *keys, uint64_t n, uint32_t shift, uint32_t mask,
                                                        uint32_t n_tiles, uint32_t *hist) {
  __shared__ uint32_t h[256];
  if (threadIdx.x < 256) h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kRsTile;
#pragma unroll
  for (uint32_t j = 0; j < kRsItems; j++) {
    const uint64_t i = t0 + (uint64_t)j * kRsThreads + threadIdx.x;
    if (i < n) atomicAdd(&h[rs_digit(keys[i], shift, mask)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 256) hist[(uint64_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

// Exclusive scan of the tile-major histogram in (digit, tile) order — every
// run's global start, tile-major: start[t][d] = sum of all counts of digits
// < d + sum of digit d's counts in tiles < t.  Three coalesced passes over
// groups of kColGroup tiles (thread = digit): group sums, group bases (one
// workgroup), per-tile prefixes inside each group.
constexpr uint32_t kColGroup = 256;
// (column walks load kColBatch rows at a time, so their round trips overlap)
constexpr uint32_t kColBatch = 16;
__global__ void __launch_bounds__(256) k_col_sums(const uint32_t *hist, uint32_t n_tiles, uint32_t *gsum) {
  const uint32_t g = blockIdx.x, d = threadIdx.x;
  const uint32_t t1 = min(n_tiles, (g + 1) * kColGroup);
  uint32_t s = 0;
  for (uint32_t t0 = g * kColGroup; t0 < t1; t0 += kColBatch) {
    uint32_t v[kColBatch];
#pragma unroll
    for (uint32_t j = 0; j < kColBatch; j++) v[j] = t0 + j < t1 ? hist[(uint64_t)(t0 + j) * 256 + d] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < kColBatch; j++) s += v[j];
  }
  gsum[(uint64_t)g * 256 + d] = s;
}
__global__ void __launch_bounds__(256) k_col_bases(uint32_t *gsum, uint32_t n_groups) {
  __shared__ uint32_t wsum[4];
  const uint32_t d = threadIdx.x;
  uint32_t run = 0;                                     // digit d's groups, in place -> exclusive
  for (uint32_t g0 = 0; g0 < n_groups; g0 += kColBatch) {
    uint32_t v[kColBatch];
#pragma unroll
    for (uint32_t j = 0; j < kColBatch; j++) v[j] = g0 + j < n_groups ? gsum[(uint64_t)(g0 + j) * 256 + d] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < kColBatch; j++) {
      if (g0 + j < n_groups) gsum[(uint64_t)(g0 + j) * 256 + d] = run;
      run += v[j];
    }
  }
  uint32_t tot;
  const uint32_t base = block_incl_scan(run, wsum, &tot) - run;   // digits < d
  for (uint32_t g = 0; g < n_groups; g++) gsum[(uint64_t)g * 256 + d] += base;
}
__global__ void __launch_bounds__(256) k_col_final(const uint32_t *hist, uint32_t n_tiles, const uint32_t *gsum,
                                                   uint32_t *start) {
  const uint32_t g = blockIdx.x, d = threadIdx.x;
  const uint32_t t1 = min(n_tiles, (g + 1) * kColGroup);
  uint32_t run = gsum[(uint64_t)g * 256 + d];
  for (uint32_t t0 = g * kColGroup; t0 < t1; t0 += kColBatch) {
    uint32_t v[kColBatch];
#pragma unroll
    for (uint32_t j = 0; j < kColBatch; j++) v[j] = t0 + j < t1 ? hist[(uint64_t)(t0 + j) * 256 + d] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < kColBatch; j++) {
      if (t0 + j < t1) start[(uint64_t)(t0 + j) * 256 + d] = run;
      run += v[j];
    }
  }
}

// Per tile: stable rank of each word among the tile's words of its digit.
// Wave w takes the tile's w-th quarter (1024 consecutive words: item j of
// lane l is word 1024 w + 64 j + l, so a wave walks its words in input
// order) and ranks them against its own LDS digit counters (cursor_bump: peer
// masks rank the lanes of one instruction, the lowest peer's returning add
// gives their base); after one
// barrier the counters become per-wave digit bases (an exclusive scan over
// the waves, thread = digit), and each word goes to LDS at (digit start in
// the tile + earlier waves' words of its digit + its rank in the wave), then
// out run by run to hist-scanned global starts.  Three barriers per tile
// (round 3's 16 block-wide rounds of 256 words took three each: 48).
struct RsSmem {
  uint64_t k[kRsTile];
  uint32_t start[256];                 // digit's first position in the sorted tile
  uint32_t gpos[256];                  // digit run's global start (scanned hist)
  uint32_t wcnt[kRsWaves][257];        // the wave's words per digit (256: past the end), then bases
  uint32_t wsum[kRsWaves];
};
constexpr uint32_t kRsWaveWords = kRsItems * 64;        // consecutive words per wave

// Tile of workgroup b: workgroups go to the 8 XCDs round-robin (b mod 8), so
// XCD x gets the contiguous tile range [x n / 8, (x + 1) n / 8) in order.
// The workgroups running together on one XCD then hold consecutive tiles,
// whose runs of one digit are adjacent in the output: the lines two runs
// share are completed in that XCD's L2 instead of being written partially
// from two XCDs.
#ifndef TFIDF_RS_XCD
#define TFIDF_RS_XCD 1
#endif
__device__ __forceinline__ uint32_t rs_tile(uint32_t b, uint32_t n) {
  if (!TFIDF_RS_XCD) return b;
  const uint32_t x = b & 7u, i = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + min(x, r) + i;
}

// LAST: write postings (and df run lengths) instead of words.
template <bool LAST>
__global__ void __launch_bounds__(kRsThreads) k_rs_scatter(const uint64_t *keys, uint64_t *out, uint64_t n,
                                                           uint32_t shift, uint32_t mask, uint32_t n_tiles,
                                                           const uint32_t *hist, const uint32_t *gstart, TermParams p) {
  __shared__ RsSmem sm;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint32_t tile = rs_tile(blockIdx.x, n_tiles);
  const uint64_t t0 = (uint64_t)tile * kRsTile;
  // the tile's digit starts: exclusive scan of its histogram over digits
  {
    const uint32_t c = tid < 256 ? hist[(uint64_t)tile * 256 + tid] : 0u;
    uint32_t tot;
    const uint32_t st = block_incl_scan(c, sm.wsum, &tot) - c;
    if (tid < 256) {
      sm.start[tid] = st;
      sm.gpos[tid] = gstart[(uint64_t)tile * 256 + tid];
#pragma unroll
      for (uint32_t w = 0; w < kRsWaves; w++) sm.wcnt[w][tid] = 0;
    }
    if (tid < kRsWaves) sm.wcnt[tid][256] = 0;
  }
  const uint64_t wb = t0 + (uint64_t)wid * kRsWaveWords;
  uint64_t kv[kRsItems];
#pragma unroll
  for (uint32_t j = 0; j < kRsItems; j++) {
    const uint64_t i = wb + (uint64_t)j * 64 + lane;
    kv[j] = i < n ? keys[i] : ~0ull;
  }
  __syncthreads();
  uint32_t dr[kRsItems];                                   // digit (9 bits) | rank in the wave << 9
  const bool full = t0 + kRsTile <= n;                     // block-uniform
#pragma unroll
  for (uint32_t j = 0; j < kRsItems; j++) {
    const bool in = wb + (uint64_t)j * 64 + lane < n;
    const uint32_t d = in ? rs_digit(kv[j], shift, mask) : 256u;
    const uint32_t r = full ? cursor_bump<8>(sm.wcnt[wid], d, lane) : cursor_bump<9>(sm.wcnt[wid], d, lane);
    dr[j] = d | (r << 9);
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t run = 0;                                      // digit tid: words of the lower waves
#pragma unroll
    for (uint32_t w = 0; w < kRsWaves; w++) {
      const uint32_t c = sm.wcnt[w][tid];
      sm.wcnt[w][tid] = run;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kRsItems; j++) {
    const uint32_t d = dr[j] & 511u;
    if (d < 256) sm.k[sm.start[d] + sm.wcnt[wid][d] + (dr[j] >> 9)] = kv[j];
  }
  __syncthreads();
  // out: sorted tile position q holds a word of digit d at global gpos[d] + (q - start[d])
  const uint64_t cnt = n - t0 < kRsTile ? n - t0 : kRsTile;
  const TermLayout ly{p.slot_bits, p.doc_bits, p.tf_bits};
#pragma unroll
  for (uint32_t j = 0; j < kRsItems; j++) {
    const uint32_t q = j * kRsThreads + tid;
    if (q < cnt) {
      const uint64_t k = sm.k[q];
      const uint32_t d = rs_digit(k, shift, mask);
      const uint64_t g = (uint64_t)sm.gpos[d] + (q - sm.start[d]);
      if (!LAST) {
        out[g] = k;
      } else {
        // the last digit is the top of the key, so the tile is in (term, doc)
        // order and each term's words are one run here: the run's first and
        // last words add -first and last + 1 to df[term]
        const uint32_t slot = (uint32_t)(k >> ly.slot_shift());
        const uint64_t doc = (k >> ly.doc_shift()) & ((1ull << ly.db) - 1);
        uint32_t tf = (uint32_t)(k >> 8) & ly.tf_esc();
        if (tf == ly.tf_esc()) {                               // rare: exact tf from the escape list
          const uint64_t key = ((uint64_t)slot << kTermDocBits) | doc;
          uint64_t a = 0, z = p.n_tesc;
          while (a < z) {
            const uint64_t m = (a + z) >> 1;
            if (p.tesc[2 * m] < key) a = m + 1; else z = m;
          }
          tf = (uint32_t)p.tesc[2 * a + 1];
        }
        out[g] = doc | ((uint64_t)((tf << 8) | (uint32_t)(k & 255u)) << 32);
        if (q == 0 || (uint32_t)(sm.k[q - 1] >> ly.slot_shift()) != slot) atomicSub(&p.df[slot], (uint32_t)g);
        if (q + 1 == cnt || (uint32_t)(sm.k[q + 1] >> ly.slot_shift()) != slot) atomicAdd(&p.df[slot], (uint32_t)g + 1);
      }
    }
  }
}

// ---------------------------------------------------------------------------

// toff (u64, C + 1 entries) from the exclusive scan of df (u32)
__global__ void k_term_toff(const uint32_t *scan, uint32_t C, uint64_t nnz, uint64_t *toff) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < C) toff[s] = scan[s];
  else if (s == C) toff[C] = nnz;
}

// scratch layout (u32 words): hist [256 tiles] | scanned hist [256 tiles] |
// scan block sums | df scan [C]
static uint64_t scan_sums_words(uint64_t n_docs, uint64_t nnz, uint32_t C) {
  const uint64_t tiles = (nnz + kRsTile - 1) / kRsTile, hist = 256 * tiles;
  const uint64_t col = 256 * ((tiles + kColGroup - 1) / kColGroup);          // column-scan group sums
  return std::max<uint64_t>((std::max<uint64_t>(std::max<uint64_t>(hist, n_docs), C) + kScanBlock - 1) / kScanBlock,
                            col) + 16;
}
// ... | tile_doc [tiles] (k_term_pairs_tiled)
static uint64_t tile_doc_offset(uint64_t n_docs, uint64_t nnz, uint32_t C) {
  const uint64_t hist = 256 * ((nnz + kRsTile - 1) / kRsTile);
  return 2 * hist + scan_sums_words(n_docs, nnz, C) + C + 16;
}
uint64_t term_invert_scratch_words(uint64_t n_docs, uint64_t nnz, uint32_t C) {
  return tile_doc_offset(n_docs, nnz, C) + (nnz + kRsTile - 1) / kRsTile + 16;
}
// Book-sized rows (SURVEY cfg 1) keep the row kernels (k_term_pairs_wide: many
// workgroups per row) and the first k_rs_hist pass; TFIDF_TERM_PAIRS_ROWS forces them (A/B)
static bool term_rows_path(const TermParams &p) {
  return knob("TFIDF_TERM_PAIRS_ROWS") != nullptr || (p.n_docs && p.nnz / p.n_docs > 2048);
}

hipError_t launch_term_pairs(const TermParams &p, hipStream_t s) {
  hipError_t e = scan_u32_excl(p.doc_nuniq, p.row_off, p.n_docs, p.scratch, s);
  if (e != hipSuccess) return e;
  if (!term_rows_path(p)) {
    const uint32_t tiles = (uint32_t)((p.nnz + kRsTile - 1) / kRsTile);
    if (!tiles) return hipGetLastError();
    uint32_t *tile_doc = p.scratch + tile_doc_offset(p.n_docs, p.nnz, p.C);
    hipLaunchKernelGGL(k_tile_docs, dim3((unsigned)((p.n_docs + 255) / 256)), dim3(256), 0, s, p.row_off, p.doc_nuniq,
                       p.n_docs, tile_doc);
    hipLaunchKernelGGL(k_term_pairs_tiled, dim3(tiles), dim3(256), 0, s, p, tile_doc, p.scratch);
    return hipGetLastError();
  }
  if (p.n_docs && p.nnz / p.n_docs > 2048) {                  // long rows: many workgroups per row
    const uint64_t avg = p.nnz / p.n_docs;
    const unsigned gy = (unsigned)std::min<uint64_t>((avg + 1023) / 1024, 64);
    const unsigned gx = (unsigned)std::min<uint64_t>(p.n_docs, 1u << 16);
    hipLaunchKernelGGL(k_term_pairs_wide, dim3(gx, gy), dim3(256), 0, s, p);
    return hipGetLastError();
  }
  const uint64_t waves = std::min<uint64_t>((p.n_docs + 3) / 4, 1ull << 18);
  if (waves) hipLaunchKernelGGL(k_term_pairs, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, p);
  return hipGetLastError();
}

// After launch_term_pairs and the host sort of the (rare) tf escape list.
hipError_t launch_term_sort(const TermParams &p, hipStream_t s) {
  hipError_t e = hipMemsetAsync(p.df, 0, (size_t)p.C * 4, s);
  if (e != hipSuccess) return e;
  const uint32_t tiles = (uint32_t)((p.nnz + kRsTile - 1) / kRsTile);
  uint32_t *hist = p.scratch, *gstart = p.scratch + (size_t)256 * tiles, *sums = gstart + (size_t)256 * tiles;
  uint32_t *df_scan = sums + scan_sums_words(p.n_docs, p.nnz, p.C);
  if (p.n_docs && p.nnz) {
    uint64_t *a = p.keys, *b = p.keys_alt;
    for (uint32_t lo = 0; lo < p.slot_bits; lo += 8) {
      const uint32_t bits = p.slot_bits - lo < 8 ? p.slot_bits - lo : 8;
      const uint32_t shift = 64 - p.slot_bits + lo, mask = (1u << bits) - 1;
      const bool last = lo + 8 >= p.slot_bits;
      if (lo > 0 || term_rows_path(p))                          // (first digit: from k_term_pairs_tiled)
        hipLaunchKernelGGL(k_rs_hist, dim3(tiles), dim3(kRsThreads), 0, s, a, p.nnz, shift, mask, tiles, hist);
      const uint32_t groups = (tiles + kColGroup - 1) / kColGroup;
      hipLaunchKernelGGL(k_col_sums, dim3(groups), dim3(256), 0, s, hist, tiles, sums);
      hipLaunchKernelGGL(k_col_bases, dim3(1), dim3(256), 0, s, sums, groups);
      hipLaunchKernelGGL(k_col_final, dim3(groups), dim3(256), 0, s, hist, tiles, sums, gstart);
      if (last)
        hipLaunchKernelGGL(k_rs_scatter<true>, dim3(tiles), dim3(kRsThreads), 0, s, a, p.post, p.nnz, shift, mask,
                           tiles, hist, gstart, p);
      else
        hipLaunchKernelGGL(k_rs_scatter<false>, dim3(tiles), dim3(kRsThreads), 0, s, a, b, p.nnz, shift, mask,
                           tiles, hist, gstart, p);
      uint64_t *t = a; a = b; b = t;
    }
  }
  // toff = exclusive scan of df
  e = scan_u32_excl(p.df, df_scan, p.C, sums, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_term_toff, dim3(p.C / 256 + 1), dim3(256), 0, s, df_scan, p.C, p.nnz, p.toff);
  return hipGetLastError();
}

}  // namespace tfidf
