// kernels_query.hip — BM25 scoring + ranking (Worker.searchIndex of the
// reference, Worker.java:222-241: IndexSearcher.search(query, MAX) with
// Lucene 9.8.0 BM25Similarity and TopScoreDocCollector), for gfx950.
//
//   score_blocks : grid (doc block, query chunk); the workgroup scores the
//                  chunk's queries one after another against its block,
//                  reusing the LDS accumulator.  For each query term (in
//                  query order) it streams that term's posting segment for
//                  the block (contiguous, coalesced u64 loads) and computes
//                  s = w - w / (1f + (float)tf * cache[norm])  in float (no
//                  contraction), accumulating (double)s per doc in LDS — the
//                  disjunction's double sum — then rounds once to float.
//                  Top-k within the block: 4-pass 8-bit radix select on the
//                  float bits, ties resolved by ascending doc via a block scan
//                  over the hit bitmap (HitQueue order).
//   merge_topk   : per query, radix select over all block candidates on the
//                  64-bit key (score bits << 32 | ~doc), then a bitonic sort
//                  in LDS -> (score desc, doc asc).
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <type_traits>

#include "tfidf_common.h"
#include "tfidf_internal.h"

namespace tfidf {

constexpr uint32_t kScoreThreads = 512;
constexpr uint32_t kDocsPerThread = kBlockDocs / kScoreThreads;  // 16

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *sh, uint32_t *total) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wid] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
  for (uint32_t w = 0; w < nw; w++) {
    uint32_t s = sh[w];
    if (w < wid) base += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// BM25Scorer.score in Java float order; volatile-free: compiled with
// -ffp-contract=off so no FMA is formed.
__device__ __forceinline__ float bm25_term(float w, uint32_t tf, float norm_inverse) {
  const float t = (float)tf * norm_inverse;
  const float u = 1.0f + t;
  const float v = w / u;
  return w - v;
}

// Radix-select step, run by one whole wave: over the 256-bin histogram taken
// from the high bin down, find the bin where the running count first reaches
// rem.  Returns the bin; *above = count in higher bins.  Lane l holds bins
// 255-4l .. 252-4l; lane prefix by DPP-free shuffles (one wave).
__device__ __forceinline__ uint32_t wave_select_bin(const uint32_t *hist, uint32_t rem, uint32_t *above) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t h[4], inc[4], run = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    h[i] = hist[255 - (4 * lane + i)];
    run += h[i];
    inc[i] = run;                                   // lane-local inclusive
  }
  uint32_t x = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  const uint32_t base = x - run;                    // exclusive over lanes
  int first = -1;
#pragma unroll
  for (int i = 3; i >= 0; i--)
    if (base + inc[i] >= rem) first = i;
  const uint64_t m = __ballot(first >= 0);
  const uint32_t src = m ? (uint32_t)__builtin_ctzll(m) : 63u;
  const uint32_t fi = (uint32_t)__shfl(first < 0 ? 0 : first, (int)src, 64);
  uint32_t cum = base + (fi ? inc[fi - 1] : 0u);    // count in bins above the selected one
  cum = (uint32_t)__shfl((int)cum, (int)src, 64);
  *above = cum;
  return 255u - (4u * src + fi);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}
// bitonic stages over the 64 lanes for sequences of `size` (descending overall)
__device__ __forceinline__ uint64_t bitonic_stages(uint64_t v, uint32_t lane, uint32_t size) {
  for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
    const uint64_t o = shfl_xor64(v, (int)stride);
    const bool desc = (lane & size) == 0, lower = (lane & stride) == 0;
    v = (lower == desc) ? max(v, o) : min(v, o);
  }
  return v;
}

// Wave-cooperative lower bound over one term's doc-ascending postings
// (term-major layout): first i in [lo, hi) with doc(post[i]) >= x.  Each step
// samples 64 evenly spaced postings, so a list of df entries takes
// ceil(log64(df)) + 1 dependent loads instead of log2(df).
__device__ __forceinline__ uint64_t wave_lower_bound(const uint64_t *post, uint64_t lo, uint64_t hi, uint32_t x) {
  const uint32_t lane = threadIdx.x & 63;
  while (hi - lo > 64) {
    const uint64_t step = (hi - lo + 63) >> 6;
    const uint64_t i = lo + lane * step;
    const bool less = i < hi && (uint32_t)post[i] < x;
    const uint32_t c = (uint32_t)__popcll(__ballot(less));   // samples are sorted: lanes [0, c) are below x
    if (c == 0) return lo;
    const uint64_t nlo = lo + (uint64_t)(c - 1) * step + 1;
    hi = min(hi, lo + (uint64_t)c * step);
    lo = nlo;
  }
  const uint64_t i = lo + lane;
  const bool less = i < hi && (uint32_t)post[i] < x;
  return lo + (uint64_t)__popcll(__ballot(less));
}

// Segment of doc block [d0, d0 + kBlockDocs) in slot's postings (whole wave).
__device__ __forceinline__ void term_block_range(const QueryParams &p, uint32_t slot, uint32_t d0, uint64_t *a,
                                                 uint64_t *z) {
  const uint64_t t0 = p.toff[slot], t1 = p.toff[slot + 1];
  const uint64_t lo = wave_lower_bound(p.post, t0, t1, d0);
  *a = lo;
  *z = wave_lower_bound(p.post, lo, t1, d0 + kBlockDocs);
}

// Posting words: term-major u64 (doc | (tf << 8 | norm) << 32), block-major
// u32 post_word (doc within the block | tf | norm; tf escapes looked up in
// the sorted escape list).  The scorers are instantiated per layout.
template <bool kTerm> using PostW = typename std::conditional<kTerm, uint64_t, uint32_t>::type;
template <bool kTerm> __device__ __forceinline__ PostW<kTerm> post_raw(const QueryParams &p, uint64_t i) {
  if constexpr (kTerm) return p.post[i];
  else return p.post32[i];
}
// posting e (index i) of the block starting at doc d0
template <bool kTerm>
__device__ __forceinline__ void post_decode(const QueryParams &p, PostW<kTerm> e, uint64_t i, uint32_t d0,
                                            uint32_t *ld, uint32_t *tf, uint32_t *nrm) {
  if constexpr (kTerm) {
    const uint32_t tfn = (uint32_t)(e >> 32);
    *ld = (uint32_t)e - d0;
    *tf = tfn >> 8;
    *nrm = tfn & 255u;
  } else {
    uint32_t t = (e >> 13) & kPostTfEsc;
    if (t == kPostTfEsc) t = csr_esc_tf(p.post_esc, p.n_post_esc, i);      // rare: tf >= 2047
    *ld = e & (kBlockDocs - 1);
    *tf = t;
    *nrm = e >> 24;
  }
}

constexpr uint32_t kQTermsFast = 4;   // query terms whose ranges / first chunk are prefetched

constexpr int kMergeWaveRegs = 32;
constexpr uint32_t kMergeWavesPerWG = 4;

// One query's merge of its per-block candidate lists by one wave (see
// k_merge_topk_wave); hist: the wave's 256-word LDS histogram, zero on entry.
__device__ __forceinline__ void merge_query_wave(const QueryParams &p, uint32_t q, uint32_t *hist) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t k = p.k, nb = p.n_blocks, nflat = nb * k;
  const uint64_t *cand = p.cand + (size_t)q * nflat;
  const uint32_t *cn = p.cand_n + (size_t)q * nb;
  const uint32_t inv = (uint32_t)((0xFFFFFFFFull + k) / k);   // f / k = umulhi(f, inv) (f < 2^11, 2 <= k <= 64)
  uint64_t kv[kMergeWaveRegs];
  uint64_t lmin = ~0ull, lmax = 0;
  uint32_t cnt = 0;
#pragma unroll
  for (int r = 0; r < kMergeWaveRegs; r++) {
    const uint32_t f = lane + 64u * r;
    kv[r] = 0;
    if (f < nflat) {
      const uint32_t b = k == 1 ? f : __umulhi(f, inv);
      if (f - b * k < cn[b]) kv[r] = cand[f];
    }
    if (kv[r]) { lmin = min(lmin, kv[r]); lmax = max(lmax, kv[r]); cnt++; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cnt += (uint32_t)__shfl_xor((int)cnt, o, 64);
    lmin = min(lmin, (uint64_t)__shfl_xor((long long)lmin, o, 64));
    lmax = max(lmax, (uint64_t)__shfl_xor((long long)lmax, o, 64));
  }
  const uint32_t M = cnt, kk = M < k ? M : k;
  uint64_t T = 1, tmask = ~0ull;                            // take (key & tmask) >= T (keys > 0)
  if (M > k) {
    int rb = 64 - __builtin_clzll(lmin ^ lmax);
    uint64_t prefix = rb < 64 ? lmax & (~0ull << rb) : 0ull;
    uint32_t rem = k;
    while (rb > 0) {
      const int wd = rb < 8 ? rb : 8, sh = rb - wd;
      const uint64_t hmask = rb < 64 ? (~0ull << rb) : 0ull;
      const uint32_t dmask = (1u << wd) - 1;
#pragma unroll
      for (int r = 0; r < kMergeWaveRegs; r++)
        if (kv[r] && (kv[r] & hmask) == prefix) atomicAdd(&hist[(uint32_t)(kv[r] >> sh) & dmask], 1u);
      uint32_t above;
      const uint32_t bin = wave_select_bin(hist, rem, &above);
      const uint32_t inbin = hist[bin];
#pragma unroll
      for (int i = 0; i < 4; i++) hist[lane + 64 * i] = 0;
      prefix |= (uint64_t)bin << sh;
      rem -= above;
      rb = sh;
      if (inbin == rem) break;
    }
    tmask = ~0ull << rb;
    T = prefix;
  }
  // gather the kk winners one per lane (lane order = flat order), sort descending
  uint64_t mine = 0;
  uint32_t base = 0;
#pragma unroll
  for (int r = 0; r < kMergeWaveRegs; r++) {
    const bool take = kv[r] && (kv[r] & tmask) >= T;
    const uint64_t m = __ballot(take);
    const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
    // lane `pos` receives this key: scatter through the LDS histogram space
    if (take) reinterpret_cast<uint64_t *>(hist)[pos & 127] = kv[r];
    base += (uint32_t)__popcll(m);
  }
  __builtin_amdgcn_wave_barrier();
  if (lane < kk) mine = reinterpret_cast<uint64_t *>(hist)[lane];
#pragma unroll
  for (uint32_t size = 2; size <= 64; size <<= 1) mine = bitonic_stages(mine, lane, size);
  if (lane < kk) {
    p.out_doc[(size_t)q * k + lane] = ~(uint32_t)(mine & 0xFFFFFFFFu);
    p.out_score[(size_t)q * k + lane] = __uint_as_float((uint32_t)(mine >> 32));
  }
  if (lane == 0) p.out_n[q] = kk;
}

// kOps: queries with MUST / MUST_NOT clauses (QueryParser operator words,
// analysis.h).  Per document: acc = the current MUST clause's double sum, then
// the SHOULD double sum; req = double sum of the MUST clauses' float scores;
// bitmaps of the current clause, of every MUST clause so far and of MUST_NOT.
template <bool kOps> struct ScoreSmem {
  double acc[kBlockDocs];
  double req[kOps ? kBlockDocs : 1];
  uint32_t grpbits[kOps ? kBlockDocs / 32 : 1];
  uint32_t reqbits[kOps ? kBlockDocs / 32 : 1];
  uint32_t notbits[kOps ? kBlockDocs / 32 : 1];
  uint64_t tlo[kQTermsFast], thi[kQTermsFast];     // absolute posting ranges of the block's segments
  uint64_t xlo, xhi;                               // range of a query term beyond the first kQTermsFast
  float tw[kQTermsFast];
  uint32_t hitbits[kBlockDocs / 32];
  float cache[256];
  uint32_t hist[256];
  uint32_t scan[16];
  uint32_t nhit, prefix, remaining, outn, smin, smax, flag;
};

// Hits are enumerated from the bitmap: thread t owns docs [16 t, 16 t + 16)
// (ascending doc order for ties).  The per-query set-up is a 1 KiB bitmap
// clear, so a chunk of queries amortises the workgroup launch, and the LDS
// footprint (66 KiB) admits two workgroups per CU (kOps: 134 KiB, one).
//
// Operator queries (kOps) follow Lucene 9.8.0's scorer shapes for the
// rewritten BooleanQuery (Boolean2ScorerSupplier): a MUST clause's score is
// its float score ((float) double sum for a nested disjunction); the required
// part is (float) of the double sum of the MUST clauses (ConjunctionScorer /
// BlockMaxConjunctionScorer); SHOULD terms add (float) of their double sum in
// float (ReqOptSumScorer) when one matches; MUST_NOT excludes (ReqExclScorer).
// Without MUST clauses a document needs a SHOULD match: the plain disjunction.
//
// kAll: all-hits mode (k == 0) as its own instantiation — its LDS sort code
// made the compiler schedule the top-k instantiation's loops worse (10 k-query
// batch: 12.4 -> 16.0 ms when they shared one kernel).
// Query arrays: device memory, or (single fused queries, inl_n > 0) the
// kernel arguments themselves (no upload before the launch).
__device__ __forceinline__ uint32_t q_off_of(const QueryParams &p, uint32_t q) {
  return p.inl_n ? (q ? p.inl_n : 0u) : p.q_off[q];
}
__device__ __forceinline__ uint32_t q_slot_of(const QueryParams &p, uint32_t j) { return p.inl_n ? p.inl_slot[j] : p.q_slot[j]; }
__device__ __forceinline__ float q_w_of(const QueryParams &p, uint32_t j) { return p.inl_n ? p.inl_w[j] : p.q_w[j]; }
__device__ __forceinline__ uint32_t q_role_of(const QueryParams &p, uint32_t j) { return p.inl_n ? p.inl_role[j] : p.q_role[j]; }
__device__ __forceinline__ uint32_t q_meta_of(const QueryParams &p, uint32_t q) { return p.inl_n ? p.inl_meta : p.q_meta[q]; }

template <bool kOps, bool kAll, bool kTerm>
__global__ void __launch_bounds__(kScoreThreads) k_score_blocks(QueryParams p) {
  __shared__ ScoreSmem<kOps> sm;
  const uint32_t tid = threadIdx.x;
  const uint32_t q0 = blockIdx.y * p.q_chunk;
  const uint32_t q1 = min(p.n_q, q0 + p.q_chunk);
  for (uint32_t i = tid; i < 256; i += blockDim.x) sm.cache[i] = p.cache[i];
  const uint32_t k = p.k;
  // grid mode: workgroup (block, query chunk); list mode (ovf_list): persistent
  // workgroups over the pairs k_score_pairs left (too many postings)
  const bool listmode = p.ovf_list != nullptr;
  const uint32_t n_it = listmode ? 0xFFFFFFFFu : (q1 > q0 ? q1 - q0 : 0u);
  for (uint32_t it = 0; it < n_it; it++) {
    uint32_t q, b;
    if (listmode) {
      const uint32_t idx = blockIdx.x + it * gridDim.x;
      if (idx >= *p.ovf_count) break;                                 // uniform
      const uint32_t pr = p.ovf_list[idx];
      q = pr / p.n_blocks;
      b = pr - q * p.n_blocks;
    } else {
      q = q0 + it;
      b = blockIdx.x;
    }
    const uint64_t d0 = (uint64_t)b * kBlockDocs;
    const uint64_t bb = p.toff ? 0 : p.bbase[b];
    const uint64_t bend = p.toff ? 0 : p.bbase[b + 1];
    const uint32_t *row = p.toff ? nullptr : p.blk + (size_t)b * p.C;
    for (uint32_t i = tid; i < kBlockDocs / 32; i += blockDim.x) {
      sm.hitbits[i] = 0;
      if (kOps) { sm.grpbits[i] = 0; sm.reqbits[i] = 0; sm.notbits[i] = 0; }
    }
    for (uint32_t i = tid; i < 256; i += blockDim.x) sm.hist[i] = 0;
    if (tid == 0) { sm.nhit = 0; sm.outn = 0; sm.smin = 0xFFFFFFFFu; sm.smax = 0; }
    __syncthreads();
    const uint32_t t0 = q_off_of(p, q), t1 = q_off_of(p, q + 1);
    const uint32_t ngroups = kOps ? (q_meta_of(p, q) & 0xFFFFu) : 0u;
    bool alive = true;                                     // kOps: a document still meets every MUST clause
    if (p.toff) {
      // term-major layout: wave j finds term j's segment for this block in the
      // term's doc-sorted list (two 64-ary searches)
      const uint32_t wv = tid >> 6;
      if (wv < t1 - t0 && wv < kQTermsFast) {
        const uint32_t slot = q_slot_of(p, t0 + wv);
        uint64_t a = 0, z = 0;
        if (slot != kInvalidSlot) term_block_range(p, slot, (uint32_t)d0, &a, &z);
        if ((tid & 63) == 0) { sm.tlo[wv] = a; sm.thi[wv] = z; sm.tw[wv] = q_w_of(p, t0 + wv); }
      }
    } else if (tid < t1 - t0 && tid < kQTermsFast) {
      // block-major layout: all terms' ranges in one round trip (thread j fetches term j)
      const uint32_t slot = q_slot_of(p, t0 + tid);
      uint64_t a = 0, z = 0;
      if (slot != kInvalidSlot) {
        a = bb + row[slot];
        z = slot + 1 < p.C ? bb + row[slot + 1] : bend;
      }
      sm.tlo[tid] = a;
      sm.thi[tid] = z;
      sm.tw[tid] = q_w_of(p, t0 + tid);
    }
    __syncthreads();
    // first chunk of every term's postings in flight before any is consumed
    PostW<kTerm> pre[kQTermsFast];
#pragma unroll
    for (uint32_t j = 0; j < kQTermsFast; j++) {
      pre[j] = 0;
      if (j < t1 - t0 && sm.tlo[j] + tid < sm.thi[j]) pre[j] = post_raw<kTerm>(p, sm.tlo[j] + tid);
    }
    uint32_t my_new = 0;
    for (uint32_t j = t0; j < t1; j++) {
      if (kOps && !alive) break;                           // uniform: no document can match any more
      const uint32_t jj = j - t0;
      const uint32_t role = kOps ? q_role_of(p, j) >> 24 : kRoleShould;
      uint64_t lo, hi;
      float w;
      if (jj < kQTermsFast) {
        lo = sm.tlo[jj];
        hi = sm.thi[jj];
        w = sm.tw[jj];
      } else {
        const uint32_t slot = q_slot_of(p, j);
        w = q_w_of(p, j);
        if (slot == kInvalidSlot) {                        // uniform
          lo = hi = 0;
        } else if (p.toff) {
          if (tid < 64) {
            uint64_t a, z;
            term_block_range(p, slot, (uint32_t)d0, &a, &z);
            if (tid == 0) { sm.xlo = a; sm.xhi = z; }
          }
          __syncthreads();
          lo = sm.xlo;
          hi = sm.xhi;
        } else {
          lo = bb + row[slot];
          hi = slot + 1 < p.C ? bb + row[slot + 1] : bend;
        }
      }
      for (uint64_t i = lo + tid; i < hi; i += blockDim.x) {
        PostW<kTerm> e;
        if (jj < kQTermsFast && i == lo + tid) {
#pragma unroll
          for (uint32_t u = 0; u < kQTermsFast; u++)
            if (u == jj) e = pre[u];
        } else {
          e = post_raw<kTerm>(p, i);
        }
        uint32_t ld, tf, nrm;
        post_decode<kTerm>(p, e, i, (uint32_t)d0, &ld, &tf, &nrm);
        const uint32_t bit = 1u << (ld & 31);
        if (kOps && role == kRoleNot) {
          atomicOr(&sm.notbits[ld >> 5], bit);
          continue;
        }
        const float sc = bm25_term(w, tf, sm.cache[nrm]);
        uint32_t *bm = (kOps && role == kRoleMust) ? sm.grpbits : sm.hitbits;
        const uint32_t old = atomicOr(&bm[ld >> 5], bit);
        if (old & bit) {
          sm.acc[ld] += (double)sc;
        } else {
          sm.acc[ld] = (double)sc;
          my_new++;
        }
      }
      __syncthreads();                                     // term order = the disjunction's sum order
      if (kOps && role == kRoleMust && (j + 1 == t1 || q_role_of(p, j + 1) != q_role_of(p, j))) {
        // end of MUST clause g: fold its float score into req for the documents
        // that met every MUST clause so far (one 32-doc word per thread)
        const uint32_t g = q_role_of(p, j) & 0xFFFFFFu;
        uint32_t rb = 0;
        if (tid < kBlockDocs / 32) {
          const uint32_t gb = sm.grpbits[tid];
          rb = g == 0 ? gb : (sm.reqbits[tid] & gb);
          for (uint32_t x = rb; x; x &= x - 1) {
            const uint32_t ld = tid * 32 + (__ffs(x) - 1);
            const double cs = (double)(float)sm.acc[ld];
            sm.req[ld] = g == 0 ? cs : sm.req[ld] + cs;
          }
          sm.reqbits[tid] = rb;
          sm.grpbits[tid] = 0;
        }
        alive = __syncthreads_or(rb != 0) != 0;
      }
    }
    if (kOps) {
      // final match set and score per document: required part, plus the
      // SHOULD part in float when one matched; MUST_NOT documents dropped
      uint32_t cnt = 0;
      if (tid < kBlockDocs / 32) {
        const uint32_t sb = sm.hitbits[tid];
        const uint32_t mb = (ngroups ? (alive ? sm.reqbits[tid] : 0u) : sb) & ~sm.notbits[tid];
        for (uint32_t x = mb; x; x &= x - 1) {
          const uint32_t b = __ffs(x) - 1, ld = tid * 32 + b;
          float sc;
          if (ngroups) {
            const float r = (float)sm.req[ld];
            sc = (sb >> b) & 1u ? r + (float)sm.acc[ld] : r;
          } else {
            sc = (float)sm.acc[ld];
          }
          sm.acc[ld] = (double)sc;
        }
        sm.hitbits[tid] = mb;
        cnt = (uint32_t)__popc(mb);
      }
      if (cnt) atomicAdd(&sm.nhit, cnt);
    } else if (my_new) {
      atomicAdd(&sm.nhit, my_new);
    }
    __syncthreads();
    const uint32_t nhit = sm.nhit;
    const uint32_t bits = (sm.hitbits[tid >> 1] >> (16 * (tid & 1))) & 0xFFFFu;
    if (kAll) {
      // all-hits mode (single query): the block's hit keys (score bits << 32 |
      // ~doc), compacted and sorted descending in LDS (bitonic over the
      // accumulator's 64 KiB) -> one sorted run per block for k_merge_runs
      uint64_t kv[kDocsPerThread];
#pragma unroll
      for (uint32_t i = 0; i < kDocsPerThread; i++) {
        const uint32_t ld = tid * kDocsPerThread + i;
        kv[i] = ((bits >> i) & 1u)
                    ? ((uint64_t)__float_as_uint((float)sm.acc[ld]) << 32) | (uint64_t)(~(uint32_t)(d0 + ld))
                    : 0ull;
      }
      uint32_t tot;
      uint32_t at = block_excl_scan((uint32_t)__popc(bits), sm.scan, &tot);   // barriers: reads of acc done
      uint64_t *keys = reinterpret_cast<uint64_t *>(sm.acc);
#pragma unroll
      for (uint32_t i = 0; i < kDocsPerThread; i++)
        if ((bits >> i) & 1u) keys[at++] = kv[i];
      uint32_t P = 2;
      while (P < nhit) P <<= 1;
      for (uint32_t i = nhit + tid; i < P; i += blockDim.x) keys[i] = 0ull;
      __syncthreads();
      for (uint32_t size = 2; size <= P; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
          for (uint32_t i = tid; i < P / 2; i += blockDim.x) {
            const uint32_t lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
            const uint64_t a = keys[lo], c = keys[hi];
            if ((lo & size) == 0 ? a < c : a > c) { keys[lo] = c; keys[hi] = a; }
          }
          __syncthreads();
        }
      }
      for (uint32_t i = tid; i < nhit; i += blockDim.x) p.hits[(size_t)b * kBlockDocs + i] = keys[i];
      if (tid == 0) p.hits_n[b] = nhit;
      __syncthreads();
      continue;
    }
    uint64_t *cand = p.cand + ((size_t)q * p.n_blocks + b) * k;
    if (nhit <= k) {
      uint32_t tot;
      uint32_t at = block_excl_scan((uint32_t)__popc(bits), sm.scan, &tot);
      for (uint32_t x = bits; x; x &= x - 1) {
        const uint32_t ld = tid * kDocsPerThread + (__ffs(x) - 1);
        cand[at++] = ((uint64_t)__float_as_uint((float)sm.acc[ld]) << 32) | (uint64_t)(~(uint32_t)(d0 + ld));
      }
      if (tid == 0) p.cand_n[(size_t)q * p.n_blocks + b] = nhit;
      __syncthreads();
      continue;
    }
    // Radix select of the k-th largest score bits, starting at the byte of the
    // highest bit on which the block's hits differ (scores share sign and
    // most exponent bits) and stopping as soon as the boundary bin holds
    // exactly the entries still needed.  Scores are converted to float bits
    // once, in place (low word of acc[ld]).
    uint32_t mn = 0xFFFFFFFFu, mx = 0;
    for (uint32_t x = bits; x; x &= x - 1) {
      const uint32_t ld = tid * kDocsPerThread + (__ffs(x) - 1);
      const uint32_t sb = __float_as_uint((float)sm.acc[ld]);
      reinterpret_cast<uint32_t *>(&sm.acc[ld])[0] = sb;
      mn = min(mn, sb);
      mx = max(mx, sb);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {                     // wave min/max, then one LDS atomic per wave
      mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    }
    if ((tid & 63) == 0 && mx) { atomicMin(&sm.smin, mn); atomicMax(&sm.smax, mx); }
    __syncthreads();
    // bits [r, 32) are common to all hits / resolved; each pass takes the next
    // (up to) 8 bits below r as the digit, so the first digit is the top 8
    // bits on which the hits differ
    const uint32_t diff = sm.smin ^ sm.smax;
    int r = diff ? 32 - __builtin_clz(diff) : 0;
    uint32_t prefix = r < 32 ? sm.smax & (0xFFFFFFFFu << r) : 0u;
    uint32_t rem = k;
    bool all_bin = false;                                  // boundary bin entirely taken
    // hist is zero here (cleared at the query start, and by wave 0 after each
    // selection), so a pass costs two barriers: histogram, selection
    while (r > 0) {
      const int w = r < 8 ? r : 8, sh = r - w;
      const uint32_t hmask = r < 32 ? (0xFFFFFFFFu << r) : 0u;
      for (uint32_t x = bits; x; x &= x - 1) {
        const uint32_t sb = reinterpret_cast<const uint32_t *>(&sm.acc[tid * kDocsPerThread + (__ffs(x) - 1)])[0];
        if ((sb & hmask) == prefix) atomicAdd(&sm.hist[(sb >> sh) & ((1u << w) - 1)], 1u);
      }
      __syncthreads();
      if (tid < 64) {
        uint32_t above;
        const uint32_t bin = wave_select_bin(sm.hist, rem, &above);
        const uint32_t inbin = sm.hist[bin];
#pragma unroll
        for (int i = 0; i < 4; i++) sm.hist[tid + 64 * i] = 0;
        if (tid == 0) {
          sm.prefix = prefix | (bin << sh);
          sm.remaining = rem - above;
          sm.flag = inbin == rem - above;
        }
      }
      __syncthreads();
      prefix = sm.prefix;
      rem = sm.remaining;
      all_bin = sm.flag != 0;
      r = sh;
      if (all_bin) break;
    }
    // T = prefix over bits [r, 32): keys above it are taken, keys in it are all
    // taken (all_bin) or, fully resolved (r = 0), ties in doc order
    const uint32_t tmask = 0xFFFFFFFFu << r;
    const uint32_t T = prefix, take_ties = all_bin ? 0xFFFFFFFFu : rem;
    uint32_t nties = 0;
    for (uint32_t x = bits; x; x &= x - 1) {
      const uint32_t ld = tid * kDocsPerThread + (__ffs(x) - 1);
      nties += (reinterpret_cast<const uint32_t *>(&sm.acc[ld])[0] & tmask) == T;
    }
    uint32_t tot;
    uint32_t tie_rank = block_excl_scan(nties, sm.scan, &tot);
    for (uint32_t x = bits; x; x &= x - 1) {
      const uint32_t ld = tid * kDocsPerThread + (__ffs(x) - 1);
      const uint32_t sb = reinterpret_cast<const uint32_t *>(&sm.acc[ld])[0];
      bool take = (sb & tmask) > T;
      if ((sb & tmask) == T) take = tie_rank++ < take_ties;
      if (take) cand[atomicAdd(&sm.outn, 1u)] = ((uint64_t)sb << 32) | (uint64_t)(~(uint32_t)(d0 + ld));
    }
    __syncthreads();
    if (tid == 0) p.cand_n[(size_t)q * p.n_blocks + b] = sm.outn;
    __syncthreads();
  }
}

// One workgroup (1024 threads) per query.  Candidates are read flat (thread t
// takes slots t, t + 1024, ... of the [block][k] candidate array) and kept in
// registers when there are at most 4 per thread; radix select from the first
// byte on which the candidates differ, stopping once the boundary bin is
// entirely needed.  Keys (score bits << 32 | ~doc) are unique.
struct MergeSmem {
  uint64_t keys[1024];
  uint32_t hist[256];
  uint64_t prefix, kmin, kmax;
  uint32_t remaining, outn, total, all_bin;
};

constexpr int kMergeRegs = 4;

__global__ void __launch_bounds__(1024) k_merge_topk(QueryParams p) {
  __shared__ MergeSmem sm;
  const uint32_t q = blockIdx.x, tid = threadIdx.x, k = p.k;
  const uint32_t nb = p.n_blocks;
  const uint64_t *cand = p.cand + (size_t)q * nb * k;
  const uint32_t *cn = p.cand_n + (size_t)q * nb;
  const uint32_t nflat = nb * k;
  if (tid == 0) { sm.total = 0; sm.outn = 0; sm.kmin = ~0ull; sm.kmax = 0; sm.all_bin = 0; }
  for (uint32_t i = tid; i < 256; i += blockDim.x) sm.hist[i] = 0;
  __syncthreads();
  uint32_t part = 0;
  for (uint32_t b = tid; b < nb; b += blockDim.x) part += cn[b];
  if (part) atomicAdd(&sm.total, part);
  auto key_at = [&](uint32_t f) -> uint64_t {
    const uint32_t b = f / k, i = f - b * k;
    return i < cn[b] ? cand[f] : 0ull;                     // 0 = empty (real keys have score bits > 0)
  };
  const bool inreg = nflat <= kMergeRegs * blockDim.x;
  uint64_t kr[kMergeRegs];
  uint64_t lmin = ~0ull, lmax = 0;
#pragma unroll
  for (int r = 0; r < kMergeRegs; r++) {
    const uint32_t f = tid + r * blockDim.x;
    kr[r] = inreg && f < nflat ? key_at(f) : 0ull;
    if (kr[r]) { lmin = min(lmin, kr[r]); lmax = max(lmax, kr[r]); }
  }
  if (!inreg)
    for (uint32_t f = tid; f < nflat; f += blockDim.x) {
      const uint64_t key = key_at(f);
      if (key) { lmin = min(lmin, key); lmax = max(lmax, key); }
    }
  if (lmax) {
    atomicMin(reinterpret_cast<unsigned long long *>(&sm.kmin), (unsigned long long)lmin);
    atomicMax(reinterpret_cast<unsigned long long *>(&sm.kmax), (unsigned long long)lmax);
  }
  __syncthreads();
  const uint32_t M = sm.total;
  const uint32_t kk = M < k ? M : k;
  uint64_t T = 0, tmask = ~0ull;                          // take (key & tmask) >= T
  if (M > k) {
    const uint64_t diff = sm.kmin ^ sm.kmax;                // != 0: keys are unique
    int rb = 64 - __builtin_clzll(diff);                    // bits [rb, 64) common / resolved
    uint64_t prefix = rb < 64 ? sm.kmax & (~0ull << rb) : 0ull;
    uint32_t rem = kk;
    while (rb > 0) {                                        // hist is zero (cleared at start / by wave 0)
      const int w = rb < 8 ? rb : 8, sh = rb - w;
      const uint64_t hmask = rb < 64 ? (~0ull << rb) : 0ull;
      const uint32_t dmask = (1u << w) - 1;
      if (inreg) {
#pragma unroll
        for (int r = 0; r < kMergeRegs; r++)
          if (kr[r] && (kr[r] & hmask) == prefix) atomicAdd(&sm.hist[(uint32_t)(kr[r] >> sh) & dmask], 1u);
      } else {
        for (uint32_t f = tid; f < nflat; f += blockDim.x) {
          const uint64_t key = key_at(f);
          if (key && (key & hmask) == prefix) atomicAdd(&sm.hist[(uint32_t)(key >> sh) & dmask], 1u);
        }
      }
      __syncthreads();
      if (tid < 64) {
        uint32_t above;
        const uint32_t bin = wave_select_bin(sm.hist, rem, &above);
        const uint32_t inbin = sm.hist[bin];
#pragma unroll
        for (int i = 0; i < 4; i++) sm.hist[tid + 64 * i] = 0;
        if (tid == 0) {
          sm.prefix = prefix | ((uint64_t)bin << sh);
          sm.remaining = rem - above;
          sm.all_bin = inbin == rem - above;
        }
      }
      __syncthreads();
      prefix = sm.prefix;
      rem = sm.remaining;
      rb = sh;
      if (sm.all_bin != 0) break;
    }
    tmask = ~0ull << rb;
    T = prefix;
  }
  if (inreg) {
#pragma unroll
    for (int r = 0; r < kMergeRegs; r++)
      if (kr[r] && (kr[r] & tmask) >= T) {
        const uint32_t pos = atomicAdd(&sm.outn, 1u);
        if (pos < 1024) sm.keys[pos] = kr[r];
      }
  } else {
    for (uint32_t f = tid; f < nflat; f += blockDim.x) {
      const uint64_t key = key_at(f);
      if (key && (key & tmask) >= T) {
        const uint32_t pos = atomicAdd(&sm.outn, 1u);
        if (pos < 1024) sm.keys[pos] = key;
      }
    }
  }
  __syncthreads();
  // bitonic sort (descending) of kk keys padded to a power of two
  uint32_t P = 1;
  while (P < kk) P <<= 1;
  for (uint32_t i = kk + tid; i < P; i += blockDim.x) sm.keys[i] = 0;
  __syncthreads();
  for (uint32_t size = 2; size <= P; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = tid; i < P; i += blockDim.x) {
        const uint32_t j = i ^ stride;
        if (j > i) {
          const bool desc = (i & size) == 0;
          const uint64_t a = sm.keys[i], c = sm.keys[j];
          if (desc ? (a < c) : (a > c)) { sm.keys[i] = c; sm.keys[j] = a; }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = tid; i < kk; i += blockDim.x) {
    const uint64_t key = sm.keys[i];
    p.out_doc[(size_t)q * k + i] = ~(uint32_t)(key & 0xFFFFFFFFu);
    p.out_score[(size_t)q * k + i] = __uint_as_float((uint32_t)(key >> 32));
  }
  if (tid == 0) p.out_n[q] = kk;
}

// ---------------------------------------------------------------------------
// Wave per (doc block, query) pair — the batched path.  A query's postings in
// one 8192-doc block are few (cfg 4: ~500), so instead of a dense 64 KiB
// accumulator and ~14 workgroup barriers per pair, one wavefront scores the
// pair into a private 1024-slot LDS hash table (doc -> double) and selects the
// block's top-k with wave-level radix passes over unique 64-bit keys
// (score bits << 32 | ~doc: (score desc, doc asc) is plain key order, so ties
// need no extra pass).  No workgroup barrier after the set-up; 12 waves per
// CU hide the LDS/HBM latencies.  Pairs with more than kPairMaxPost postings
// are appended to ovf_list and left to k_score_blocks (list mode).  Term order per document is
// the query order (the wave processes terms in sequence), so each score is the
// same double sum as the dense path.
constexpr uint32_t kPairSlots = 1024;
constexpr uint32_t kPairMaxPost = 768;
constexpr uint32_t kPairWaves = kPairWavesPerWG;
constexpr uint32_t kPairEmpty = 0xFFFFFFFFu;

struct PairSmem {
  uint32_t key[kPairWaves][kPairSlots];           // doc - d0 per slot (kPairEmpty = free)
  double val[kPairWaves][kPairSlots];             // score sum per slot
  uint32_t hist[kPairWaves][256];
  uint32_t list[kPairWaves][kPairMaxPost / 2];    // claimed slots (u16), in claim order
  float cache[256];
};

template <bool kTerm>
__global__ void __launch_bounds__(kPairWaves * 64) k_score_pairs(QueryParams p) {
  __shared__ PairSmem sm;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) sm.cache[i] = p.cache[i];
  for (uint32_t i = lane; i < 256; i += 64) sm.hist[w][i] = 0;
  __syncthreads();
  uint32_t *key = sm.key[w];
  double *val = sm.val[w];
  uint32_t *hist = sm.hist[w];
  const uint32_t nb = p.n_blocks, k = p.k;
  const uint64_t npairs = (uint64_t)p.n_q * nb;
  for (uint64_t pr = (uint64_t)blockIdx.x * kPairWaves + w; pr < npairs; pr += (uint64_t)gridDim.x * kPairWaves) {
    const uint32_t q = (uint32_t)(pr / nb), b = (uint32_t)(pr - (uint64_t)q * nb);
    const uint32_t d0 = b * kBlockDocs;
    const uint32_t t0 = p.q_off[q], t1 = p.q_off[q + 1];
    if (p.q_meta && p.q_meta[q]) {                        // MUST / MUST_NOT clauses: k_score_blocks<true>
      if (lane == 0) p.ovf2_list[atomicAdd(p.ovf2_count, 1u)] = (uint32_t)pr;
      continue;
    }
    // ranges of the first 64 terms (lane j holds term j); longer queries go dense
    uint64_t a = 0, z = 0;
    float tw = 0.f;
    const uint32_t nt = t1 - t0;
    if (nt > 64) { if (lane == 0) p.ovf_list[atomicAdd(p.ovf_count, 1u)] = (uint32_t)pr; continue; }
    if (p.toff) {
      for (uint32_t j = 0; j < nt; j++) {
        const uint32_t slot = p.q_slot[t0 + j];
        uint64_t ja = 0, jz = 0;
        if (slot != kInvalidSlot) term_block_range(p, slot, d0, &ja, &jz);
        if (lane == j) { a = ja; z = jz; }
      }
    } else if (lane < nt) {
      const uint32_t slot = p.q_slot[t0 + lane];
      if (slot != kInvalidSlot) {
        const uint32_t *row = p.blk + (size_t)b * p.C;
        const uint64_t bb = p.bbase[b];
        a = bb + row[slot];
        z = slot + 1 < p.C ? bb + row[slot + 1] : p.bbase[b + 1];
      }
    }
    if (lane < nt) tw = p.q_w[t0 + lane];
    uint32_t P = (uint32_t)(z - a);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) P += (uint32_t)__shfl_xor((int)P, o, 64);
    uint64_t *cand = p.cand + pr * k;
    if (P > kPairMaxPost) { if (lane == 0) p.ovf_list[atomicAdd(p.ovf_count, 1u)] = (uint32_t)pr; continue; }
    if (P == 0) { if (lane == 0) p.cand_n[pr] = 0; continue; }
    // the first two 64-posting chunks of the first kQTermsFast terms: all in
    // flight before the table is cleared (one HBM latency for a typical pair)
    PostW<kTerm> pre[kQTermsFast][2];
#pragma unroll
    for (uint32_t j = 0; j < kQTermsFast; j++) {
      const uint64_t ja = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a, j);
      const uint64_t jz = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(z >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)z, j);
#pragma unroll
      for (uint32_t c = 0; c < 2; c++) {
        const uint64_t i = ja + lane + 64 * c;
        pre[j][c] = (j < nt && i < jz) ? post_raw<kTerm>(p, i) : 0;
      }
    }
    {
      uint4 *kw = reinterpret_cast<uint4 *>(key);
#pragma unroll
      for (int i = 0; i < (int)(kPairSlots / 4 / 64); i++)
        kw[lane + 64 * i] = make_uint4(kPairEmpty, kPairEmpty, kPairEmpty, kPairEmpty);
    }
    uint32_t nhit = 0;
    uint32_t nlist = 0;                                          // wave-uniform count of claimed slots
    uint16_t *list = reinterpret_cast<uint16_t *>(sm.list[w]);
    // insert one posting per lane (inactive lanes: e = 0 and act = false);
    // claimed slots are appended to the wave's hit list
    auto insert = [&](PostW<kTerm> e, bool act, float wj, uint64_t i) {
      uint32_t claimed = kPairEmpty;
      if (act) {
        uint32_t ld, tf, nrm;
        post_decode<kTerm>(p, e, i, d0, &ld, &tf, &nrm);
        const float sc = bm25_term(wj, tf, sm.cache[nrm]);
        uint32_t slot = (ld * 0x9E3779B1u) >> 22;
        for (;;) {
          const uint32_t old = atomicCAS(&key[slot], kPairEmpty, ld);
          if (old == kPairEmpty) { val[slot] = (double)sc; claimed = slot; break; }
          if (old == ld) { val[slot] += (double)sc; break; }
          slot = (slot + 1) & (kPairSlots - 1);
        }
      }
      const bool c = claimed != kPairEmpty;
      const uint64_t m = __ballot(c);
      if (c) list[nlist + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = (uint16_t)claimed;
      nlist += (uint32_t)__popcll(m);
    };
    for (uint32_t j = 0; j < nt; j++) {
      const uint64_t ja = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a, j);
      const uint64_t jz = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(z >> 32), j) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)z, j);
      const float wj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), j));
      uint64_t i0 = ja;
      if (j < kQTermsFast) {
        PostW<kTerm> e0 = 0, e1 = 0;
#pragma unroll
        for (uint32_t u = 0; u < kQTermsFast; u++)
          if (u == j) { e0 = pre[u][0]; e1 = pre[u][1]; }
        insert(e0, ja + lane < jz, wj, ja + lane);
        if (ja + 64 < jz) insert(e1, ja + 64 + lane < jz, wj, ja + 64 + lane);     // uniform
        i0 = ja + 128;
      }
      // remaining chunks, four loads in flight per step
      for (; i0 < jz; i0 += 256) {
        PostW<kTerm> e[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint64_t i = i0 + 64 * u + lane;
          e[u] = i < jz ? post_raw<kTerm>(p, i) : 0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (i0 + 64 * u < jz) insert(e[u], i0 + 64 * u + lane < jz, wj, i0 + 64 * u + lane);
      }
    }
    nhit = nlist;
    // this lane's hits as selection keys, in registers
    constexpr int kPer = (int)((kPairMaxPost + 63) / 64);
    uint64_t kv[kPer];
    uint64_t kmin = ~0ull, kmax = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const uint32_t idx = lane + 64 * u;
      kv[u] = 0;
      if (idx < nhit) {
        const uint32_t slot = list[idx];
        kv[u] = ((uint64_t)__float_as_uint((float)val[slot]) << 32) | (uint64_t)(~(d0 + key[slot]));
        kmin = min(kmin, kv[u]);
        kmax = max(kmax, kv[u]);
      }
    }
    uint64_t T = 0, tmask = ~0ull;                         // take (key & tmask) >= T
    if (nhit > k) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        kmin = min(kmin, (uint64_t)__shfl_xor((long long)kmin, o, 64));
        kmax = max(kmax, (uint64_t)__shfl_xor((long long)kmax, o, 64));
      }
      int rb = 64 - __builtin_clzll(kmin ^ kmax);          // keys unique and nhit > k >= 1: kmin != kmax
      uint64_t prefix = rb < 64 ? kmax & (~0ull << rb) : 0ull;
      uint32_t rem = k;
      while (rb > 0) {
        const int wd = rb < 8 ? rb : 8, sh = rb - wd;
        const uint64_t hmask = rb < 64 ? (~0ull << rb) : 0ull;
        const uint32_t dmask = (1u << wd) - 1;
#pragma unroll
        for (int u = 0; u < kPer; u++)
          if (kv[u] && (kv[u] & hmask) == prefix) atomicAdd(&hist[(uint32_t)(kv[u] >> sh) & dmask], 1u);
        uint32_t above;
        const uint32_t bin = wave_select_bin(hist, rem, &above);
        const uint32_t inbin = hist[bin];
#pragma unroll
        for (int i = 0; i < 4; i++) hist[lane + 64 * i] = 0;
        prefix |= (uint64_t)bin << sh;
        rem -= above;
        rb = sh;
        if (inbin == rem) break;
      }
      tmask = ~0ull << rb;
      T = prefix;
    }
    // write the taken keys (wave-compacted)
    uint32_t base = 0;
#pragma unroll
    for (int u = 0; u < kPer; u++) {
      const bool take = kv[u] && (kv[u] & tmask) >= T;
      const uint64_t m = __ballot(take);
      if (take) cand[base + (uint32_t)__popcll(m & ((1ull << lane) - 1))] = kv[u];
      base += (uint32_t)__popcll(m);
    }
    if (lane == 0) p.cand_n[pr] = base;
  }
}

// ---------------------------------------------------------------------------
// Workgroup per (query, doc-block range) unit — the batched top-k path for
// heavy plain disjunctions with k <= 64 (cfg 4, block-major postings; the
// light queries take k_score_wunits).  The host cuts each query into units of
// about T/4096 postings (heavy queries into several block ranges).  Per block
// of the unit, for each query term in query order, the 512 threads add the
// term's block segment into a dense LDS accumulator of doubles: a document's
// first touch (its bit in `bits`, set by the atomic that tests it) stores the
// term score, later terms add to it — the disjunction's double sum in query
// order, terms separated by a barrier.  Each wave then walks its quarter of
// the block's touched documents in doc order, rounds the sums to float, keys
// them (score bits << 32 | ~doc) and keeps the ones above its running k-th
// best key in a lane-held sorted top-k list (lane j = j-th best); once that
// key's score exceeds the lightest term's weight, documents only that term
// touched are not walked at all (`obits`).  No per-block selection pass, no
// candidate array per (query, block) pair, no hash probing.  At the unit end
// wave 0 merges the four lists and writes them as the candidates of pair
// (q, b0) (cand_n = 0 for the unit's other blocks); k_merge_topk orders each
// query's candidates (several units for a split query).
#ifndef TFIDF_UNIT_THREADS
#define TFIDF_UNIT_THREADS 512   // 8 waves: 4 per SIMD at two workgroups per CU (256 threads: batch device 6.06 ms, 512: 5.81)
#endif
constexpr uint32_t kUnitThreads = TFIDF_UNIT_THREADS;
constexpr uint32_t kUnitWaves = kUnitThreads / 64;
// hit scan: wave w walks bit words [w, w + 1) * kUnitScanWords, kUnitLanesPerWord
// lanes per word (each its share of the word's bits)
constexpr uint32_t kUnitScanWords = kBlockDocs / 32 / kUnitWaves;
constexpr uint32_t kUnitLanesPerWord = 64 / kUnitScanWords;
static_assert(kUnitScanWords * kUnitWaves == kBlockDocs / 32 && kUnitLanesPerWord * kUnitScanWords == 64, "scan layout");
#ifndef TFIDF_UNIT_U
#define TFIDF_UNIT_U 4
#endif
#ifndef TFIDF_UNIT_PRE
#define TFIDF_UNIT_PRE 4
#endif
constexpr uint32_t kUnitU = TFIDF_UNIT_U;      // postings per thread in flight
constexpr uint32_t kUnitPre = TFIDF_UNIT_PRE;  // query terms whose first chunk is prefetched per block

struct UnitSmem {
  double acc[kBlockDocs];                      // valid where bits is set
  uint32_t bits[kBlockDocs / 32];              // touched documents of the block
  uint32_t obits[kBlockDocs / 32];             // touched by a term other than the lightest one
  float cache[256];
  uint64_t seg_a[2][64], seg_z[2][64];         // block segment of each query term (double-buffered)
  float tw[64];
  uint64_t lists[kUnitWaves][64];
  unsigned long long thr;                      // max of the waves' k-th keys: a bound for the unit's k-th key
  uint32_t unit, light;                        // the query term of least weight (BM25 bound of its score)
};

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, 1, 64), hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), 1, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Insert the candidate keys of the lanes in cm (all above theta when cm was
// taken) into the wave's sorted list tk (lane j = j-th largest key, 0 = empty);
// theta = the k-th key (0 until k are held).  A few candidates: one at a time
// (shift-insert); many (a list filling up): bitonic sort of the candidates and
// a bitonic merge with the list (top 64 of the union).
__device__ __forceinline__ void topk_insert(uint64_t cm, uint64_t key, uint64_t &tk, uint64_t &theta, uint32_t k,
                                            uint32_t lane) {
  if (__popcll(cm) > 4) {
    uint64_t v = ((cm >> lane) & 1ull) ? key : 0ull;
#pragma unroll
    for (uint32_t size = 2; size <= 64; size <<= 1) v = bitonic_stages(v, lane, size);
    tk = max(tk, shfl64(v, 63 - (int)lane));                    // bitonic: the top 64 of both lists
    tk = bitonic_stages(tk, lane, 64);
    theta = readlane64(tk, k - 1);
    return;
  }
  while (cm) {
    const uint32_t l = (uint32_t)__builtin_ctzll(cm);
    cm &= cm - 1;
    const uint64_t ck = readlane64(key, l);
    if (ck <= theta) continue;                                  // wave-uniform
    const uint32_t pos = (uint32_t)__popcll(__ballot(tk > ck));
    const uint64_t up = shfl_up64(tk);
    tk = lane > pos ? up : (lane == pos ? ck : tk);
    theta = readlane64(tk, k - 1);
  }
}

__global__ void __launch_bounds__(kUnitThreads) k_score_units(QueryParams p, const uint4 *units, uint32_t n_units,
                                                                 uint32_t *unit_ctr) {
  __shared__ UnitSmem sm;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
  for (uint32_t i = tid; i < 256; i += kUnitThreads) sm.cache[i] = p.cache[i];
  for (uint32_t i = tid; i < kBlockDocs / 32; i += kUnitThreads) sm.bits[i] = sm.obits[i] = 0;
  const uint32_t nb = p.n_blocks, k = p.k, C = p.C;
  for (;;) {
    if (tid == 0) {
      sm.unit = atomicAdd(unit_ctr, 1u);
      sm.thr = 0;
    }
    __syncthreads();                                            // also: the previous unit is finished
    const uint32_t u = sm.unit;
    if (u >= n_units) break;
    const uint4 un = units[u];
    const uint32_t q = un.x, b0 = un.y, b1 = un.z;
    const uint32_t t0 = p.q_off[q], nt = p.q_off[q + 1] - t0;  // <= 64 (host)
    uint32_t slot = kInvalidSlot;
    float tw = 0.f;
    if (tid < nt) {
      slot = p.q_slot[t0 + tid];
      tw = p.q_w[t0 + tid];
      sm.tw[tid] = tw;
    }
    if (wid == 0) {                                             // the lightest term (least BM25 weight)
      const uint32_t wb = lane < nt ? __float_as_uint(tw) : 0xFFFFFFFFu;   // weights > 0: bit order
      uint32_t m = wb;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o, 64));
      const uint64_t eq = __ballot(wb == m);
      if (lane == 0) sm.light = (uint32_t)__builtin_ctzll(eq);
    }
    // block segment of term tid (block-major: bbase[b] + blk[b][slot] ..)
    auto segment = [&](uint32_t b, uint64_t *a, uint64_t *z) {
      *a = *z = 0;
      if (slot != kInvalidSlot) {
        const uint32_t *row = p.blk + (size_t)b * C;
        const uint64_t bb = p.bbase[b];
        *a = bb + row[slot];
        *z = slot + 1 < C ? bb + row[slot + 1] : p.bbase[b + 1];
      }
    };
    // pipeline: at the top of block b, seg[b & 1] = segments of b and seg[(b + 1) & 1]
    // = segments of b + 1; pre = block b's first chunks (loaded during block b - 1).
    // Block b issues the segment loads of b + 2 and the first chunks of b + 1.
    const uint32_t bend = nt ? b1 : b0;                         // a query without terms has no hits
    if (tid < nt) {
      uint64_t a, z;
      segment(b0, &a, &z);
      sm.seg_a[b0 & 1][tid] = a;
      sm.seg_z[b0 & 1][tid] = z;
      if (b0 + 1 < bend) {
        segment(b0 + 1, &a, &z);
        sm.seg_a[(b0 + 1) & 1][tid] = a;
        sm.seg_z[(b0 + 1) & 1][tid] = z;
      }
    }
    __syncthreads();
    // first chunk of the first kUnitPre terms of block b from seg[par]
    auto prefetch = [&](uint32_t par, uint32_t (&pre)[kUnitPre][kUnitU]) {
#pragma unroll
      for (uint32_t j = 0; j < kUnitPre; j++) {
        const uint64_t a = j < nt ? sm.seg_a[par][j] : 0ull, z = j < nt ? sm.seg_z[par][j] : 0ull;
#pragma unroll
        for (int v = 0; v < (int)kUnitU; v++) {
          const uint64_t i = a + v * kUnitThreads + tid;
          pre[j][v] = i < z ? p.post32[i] : 0u;
        }
      }
    };
    uint32_t pre[kUnitPre][kUnitU];
    if (b0 < bend) prefetch(b0 & 1, pre);
    uint64_t tk = 0, theta = 0;
    for (uint32_t b = b0; b < bend; b++) {
      const uint32_t d0 = b * kBlockDocs, par = b & 1;
      __syncthreads();                                          // previous scan done; segments of b + 1 visible
      uint64_t na = 0, nz = 0;                                  // segments of b + 2, loads in flight
      if (tid < nt && b + 2 < bend) segment(b + 2, &na, &nz);
      uint32_t npre[kUnitPre][kUnitU];                          // first chunks of b + 1, loads in flight
      if (b + 1 < bend) prefetch(par ^ 1, npre);
      for (uint32_t j = 0; j < nt; j++) {
        const uint64_t a = sm.seg_a[par][j], z = sm.seg_z[par][j];
        const float wj = sm.tw[j];
        const bool other = j != sm.light;
        for (uint64_t c0 = a; c0 < z; c0 += kUnitThreads * kUnitU) {
          uint32_t e[kUnitU];
          if (c0 == a && j < kUnitPre) {
#pragma unroll
            for (int v = 0; v < (int)kUnitU; v++) {
              e[v] = pre[0][v];
#pragma unroll
              for (uint32_t jj = 1; jj < kUnitPre; jj++) e[v] = j == jj ? pre[jj][v] : e[v];
            }
          } else {
#pragma unroll
            for (int v = 0; v < (int)kUnitU; v++) {
              const uint64_t i = c0 + v * kUnitThreads + tid;
              e[v] = i < z ? p.post32[i] : 0u;
            }
          }
#pragma unroll
          for (int v = 0; v < (int)kUnitU; v++) {
            const uint64_t i = c0 + v * kUnitThreads + tid;
            if (i < z) {
              uint32_t ld, tf, nrm;
              post_decode<false>(p, e[v], i, d0, &ld, &tf, &nrm);
              const float sc = bm25_term(wj, tf, sm.cache[nrm]);
              // acc[ld] is valid where bits has ld (set by an earlier term of this
              // block): first touch stores the term score, later ones add to it
              const uint32_t bm = 1u << (ld & 31);
              if (j == 0) {
                sm.acc[ld] = (double)sc;
                atomicOr(&sm.bits[ld >> 5], bm);
              } else {
                const uint32_t ob = atomicOr(&sm.bits[ld >> 5], bm);
                sm.acc[ld] = (ob & bm) ? sm.acc[ld] + (double)sc : (double)sc;
              }
              if (other) atomicOr(&sm.obits[ld >> 5], bm);
            }
          }
        }
        __syncthreads();                                        // term j's sums land before term j + 1's
      }
      if (tid < nt && b + 2 < bend) {                           // block b's segment slots are free now
        sm.seg_a[par][tid] = na;
        sm.seg_z[par][tid] = nz;
      }
#pragma unroll
      for (uint32_t j = 0; j < kUnitPre; j++)
#pragma unroll
        for (int v = 0; v < (int)kUnitU; v++) pre[j][v] = npre[j][v];
      // wave wid scans documents [32 kUnitScanWords wid, + 32 kUnitScanWords): kUnitLanesPerWord lanes per bit word
      // two hits per lane per step (both LDS round trips in flight); no key at
      // or below another wave's k-th key (sm.thr, read once per block) can win
      // Once the k-th key's score exceeds the lightest term's weight w_l, a
      // document touched by that term alone (score <= w_l: a BM25 term score
      // never exceeds its weight) cannot enter the top-k: walk the documents
      // some other term touched (obits) only.  Heavy queries are a frequent,
      // low-idf term plus rarer ones: most hits are skipped unread.  (Skipping
      // that term's postings themselves was measured slower: 5.7 -> 6.3 ms at
      // cfg 4 — a wave of its postings almost always holds a few to score.)
      const uint32_t wi = wid * kUnitScanWords + lane / kUnitLanesPerWord;
      constexpr uint32_t kLaneBits = 32 / kUnitLanesPerWord;
      const uint32_t lmask = kUnitLanesPerWord == 1 ? 0xFFFFFFFFu
                                                    : ((1u << kLaneBits) - 1u) << (kLaneBits * (lane % kUnitLanesPerWord));
      uint64_t th = max(theta, (uint64_t)sm.thr);
      const uint64_t th_in = th;
      const bool prune = nt > 1 && sm.tw[sm.light] < __uint_as_float((uint32_t)(th >> 32));
      uint32_t wb = (prune ? sm.obits[wi] : sm.bits[wi]) & lmask;
      if (lane % kUnitLanesPerWord == 0) {                      // after the word's lanes read it (wave order)
        sm.bits[wi] = 0;
        sm.obits[wi] = 0;
      }
      while (__any(wb != 0)) {
        uint32_t x[2];
        bool has[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          has[h] = wb != 0;
          x[h] = wi * 32 + (has[h] ? (uint32_t)__builtin_ctz(wb) : 0u);
          wb &= wb - 1;
        }
        double v[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          v[h] = has[h] ? sm.acc[x[h]] : 0.0;
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const uint64_t key = has[h] ? ((uint64_t)__float_as_uint((float)v[h]) << 32) | (uint64_t)(~(d0 + x[h])) : 0ull;
          const uint64_t cm = __ballot(key > th);
          if (cm) {
            topk_insert(cm, key, tk, theta, k, lane);
            th = max(th, theta);
          }
        }
      }
      if (lane == 0 && th > th_in) atomicMax(&sm.thr, (unsigned long long)th);
    }
    // merge the waves' lists (wave 0) and write the unit's candidates
    sm.lists[wid][lane] = lane < k ? tk : 0ull;
    __syncthreads();
    if (wid == 0) {
#pragma unroll
      for (uint32_t w = 1; w < kUnitWaves; w++) {
        const uint64_t key = sm.lists[w][lane];
        topk_insert(__ballot(key > theta), key, tk, theta, k, lane);
      }
      const bool has = lane < k && tk != 0;
      const uint32_t n = (uint32_t)__popcll(__ballot(has));
      const size_t pr = (size_t)q * nb + b0;
      if (has) p.cand[pr * k + lane] = tk;
      if (lane == 0) p.cand_n[pr] = n;
    }
    for (uint32_t b = b0 + 1 + tid; b < b1; b += kUnitThreads) p.cand_n[(size_t)q * nb + b] = 0;
  }
}

hipError_t launch_score_units(const QueryParams &p, const uint4 *units, uint32_t n_units, uint32_t *unit_ctr, int grid,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_score_units, dim3(grid), dim3(kUnitThreads), 0, s, p, units, n_units, unit_ctr);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Wave per (query, doc-block range) unit — the light queries of a batch
// (few postings per block; the host sends queries averaging more than
// kWunitLightPost postings per block to k_score_units).  Per block the wave
// inserts each term's segment (query order) into its private 1024-slot LDS
// hash table (doc -> double sum, as k_score_pairs), then walks the table's
// occupied slots (round 6; a claim list before): keys above the running k-th
// best go into the lane-held top-k list (topk_insert), and every slot is reset
// on the way — no separate table clear, no per-block selection, no candidate
// array per (query, block).  A block with
// more than kWunitPassPost postings is done in 16 passes over doc sub-ranges
// of 512 documents (at most 512 distinct documents per pass, so the table
// never fills).  The next block's segments and first posting chunks are
// loaded while the current block's hits are walked.
constexpr uint32_t kWunitWaves = kPairWavesPerWG;
constexpr uint32_t kWunitPassPost = 700;

struct WunitSmem {
  uint32_t key[kWunitWaves][kPairSlots];          // doc - d0 per slot (kPairEmpty = free)
  double val[kWunitWaves][kPairSlots];
  float cache[256];
};

__global__ void __launch_bounds__(kWunitWaves * 64) k_score_wunits(QueryParams p, const uint4 *units, uint32_t n_units,
                                                                      uint32_t *unit_ctr) {
  __shared__ WunitSmem sm;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) sm.cache[i] = p.cache[i];
  uint32_t *key = sm.key[w];
  double *val = sm.val[w];
  {
    uint4 *kw = reinterpret_cast<uint4 *>(key);
#pragma unroll
    for (int i = 0; i < (int)(kPairSlots / 4 / 64); i++)
      kw[lane + 64 * i] = make_uint4(kPairEmpty, kPairEmpty, kPairEmpty, kPairEmpty);
  }
  __syncthreads();
  const uint32_t nb = p.n_blocks, k = p.k, C = p.C;
  for (;;) {
    uint32_t u = 0;
    if (lane == 0) u = atomicAdd(unit_ctr, 1u);
    u = (uint32_t)__builtin_amdgcn_readfirstlane((int)u);
    if (u >= n_units) break;
    const uint4 un = units[u];
    const uint32_t q = un.x, b0 = un.y, b1 = un.z;
    const uint32_t t0 = p.q_off[q], nt = p.q_off[q + 1] - t0;  // <= 64 (host)
    uint32_t slot = kInvalidSlot;
    float tw = 0.f;
    if (lane < nt) {
      slot = p.q_slot[t0 + lane];
      tw = p.q_w[t0 + lane];
    }
    auto segment = [&](uint32_t b, uint64_t *a, uint64_t *z) {
      *a = *z = 0;
      if (lane < nt && slot != kInvalidSlot) {
        const uint32_t *row = p.blk + (size_t)b * C;
        const uint64_t bb = p.bbase[b];
        *a = bb + row[slot];
        *z = slot + 1 < C ? bb + row[slot + 1] : p.bbase[b + 1];
      }
    };
    // first two 64-posting chunks of the first kQTermsFast terms of a block
    auto prefetch = [&](uint64_t a, uint64_t z, uint32_t (&pre)[kQTermsFast][2]) {
#pragma unroll
      for (uint32_t j = 0; j < kQTermsFast; j++) {
        const uint64_t ja = readlane64(a, j), jz = readlane64(z, j);
#pragma unroll
        for (uint32_t c = 0; c < 2; c++) {
          const uint64_t i = ja + lane + 64 * c;
          pre[j][c] = i < jz ? p.post32[i] : 0u;
        }
      }
    };
    const uint32_t bend = nt ? b1 : b0;
    uint64_t a = 0, z = 0, na = 0, nz = 0;
    uint32_t pre[kQTermsFast][2];
    if (b0 < bend) {
      segment(b0, &a, &z);
      if (b0 + 1 < bend) segment(b0 + 1, &na, &nz);
      prefetch(a, z, pre);
    }
    uint64_t tk = 0, theta = 0;
    for (uint32_t b = b0; b < bend; b++) {
      const uint32_t d0 = b * kBlockDocs;
      uint32_t P = (uint32_t)(z - a);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) P += (uint32_t)__shfl_xor((int)P, o, 64);
      const uint32_t np = P > kWunitPassPost ? 16u : 1u;          // 16 passes: 512 documents each
      const uint32_t rsh = np == 1 ? 13u : 9u;
      for (uint32_t ps = 0; ps < np; ps++) {
        // N postings per lane of one term (distinct documents): their first
        // table probes (CAS) all issued before any result is used — one LDS
        // round trip per N postings instead of per posting — then the rare
        // collisions probe on one at a time
        auto insert = [&](auto const &e, auto const &in, float wj, uint64_t i0, uint32_t stride) {
          constexpr int N = sizeof(e) / sizeof(e[0]);
          uint32_t ld[N], s[N], old[N];
          float sc[N];
          bool act[N];
#pragma unroll
          for (int v = 0; v < N; v++) {
            act[v] = false;
            ld[v] = 0;
            s[v] = 0;
            sc[v] = 0.f;
            if (in[v]) {
              uint32_t tf, nrm;
              post_decode<false>(p, e[v], i0 + (uint64_t)stride * v, d0, &ld[v], &tf, &nrm);
              if ((ld[v] >> rsh) == ps) {
                sc[v] = bm25_term(wj, tf, sm.cache[nrm]);
                s[v] = (ld[v] * 0x9E3779B1u) >> 22;
                act[v] = true;
              }
            }
          }
#pragma unroll
          for (int v = 0; v < N; v++) old[v] = act[v] ? atomicCAS(&key[s[v]], kPairEmpty, ld[v]) : 0u;
#pragma unroll
          for (int v = 0; v < N; v++) {
            if (act[v]) {
              uint32_t o = old[v], sl = s[v];
              for (;;) {
                if (o == kPairEmpty) { val[sl] = (double)sc[v]; break; }   // claimed
                if (o == ld[v]) { val[sl] += (double)sc[v]; break; }       // found
                sl = (sl + 1) & (kPairSlots - 1);
                o = atomicCAS(&key[sl], kPairEmpty, ld[v]);
              }
            }
          }
        };
        for (uint32_t j = 0; j < nt; j++) {
          const uint64_t ja = readlane64(a, j), jz = readlane64(z, j);
          const float wj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tw), (int)j));
          uint64_t i0 = ja;
          if (ps == 0 && j < kQTermsFast) {
            uint32_t e2[2] = {pre[0][0], pre[0][1]};
#pragma unroll
            for (uint32_t jj = 1; jj < kQTermsFast; jj++)
              if (jj == j) { e2[0] = pre[jj][0]; e2[1] = pre[jj][1]; }
            const bool in2[2] = {ja + lane < jz, ja + 64 + lane < jz};
            insert(e2, in2, wj, ja + lane, 64);
            i0 = ja + 128;
          }
          for (; i0 < jz; i0 += 256) {
            uint32_t e[4];
            bool in4[4];
#pragma unroll
            for (int v = 0; v < 4; v++) {
              const uint64_t i = i0 + 64 * v + lane;
              in4[v] = i < jz;
              e[v] = in4[v] ? p.post32[i] : 0u;
            }
            insert(e, in4, wj, i0 + lane, 64);
          }
        }
        if (ps + 1 == np) {                                       // next block's loads in flight during the walk
          a = na;
          z = nz;
          if (b + 2 < bend) segment(b + 2, &na, &nz);
          if (b + 1 < bend) prefetch(a, z, pre);
        }
        // walk the table itself: lane l owns slots [16 l, 16 l + 16), read as
        // four 16 B pieces in an order rotated by l / 2 (conflict-free), then
        // its occupied slots one per step; each is reset as it is read.  No
        // claim list: the workgroup's LDS is 25 KiB, six per CU instead of five
        uint32_t occ = 0;
        {
          const uint4 *kq = reinterpret_cast<const uint4 *>(key + 16 * lane);
#pragma unroll
          for (uint32_t q = 0; q < 4; q++) {
            const uint32_t qq = (q + (lane >> 1)) & 3u;
            const uint4 t = kq[qq];
            occ |= ((uint32_t)(t.x != kPairEmpty) | ((uint32_t)(t.y != kPairEmpty) << 1) |
                    ((uint32_t)(t.z != kPairEmpty) << 2) | ((uint32_t)(t.w != kPairEmpty) << 3)) << (4 * qq);
          }
        }
        while (__any(occ != 0)) {
          uint64_t kv = 0;
          if (occ) {
            const uint32_t sl = 16 * lane + (uint32_t)__builtin_ctz(occ);
            occ &= occ - 1;
            const uint32_t ld = key[sl];
            kv = ((uint64_t)__float_as_uint((float)val[sl]) << 32) | (uint64_t)(~(d0 + ld));
            key[sl] = kPairEmpty;
          }
          topk_insert(__ballot(kv > theta), kv, tk, theta, k, lane);
        }
      }
    }
    const bool has = lane < k && tk != 0;
    const uint32_t n = (uint32_t)__popcll(__ballot(has));
    const size_t pr = (size_t)q * nb + b0;
    if (has) p.cand[pr * k + lane] = tk;
    if (lane == 0) p.cand_n[pr] = n;
    for (uint32_t b = b0 + 1 + lane; b < b1; b += 64) p.cand_n[(size_t)q * nb + b] = 0;
  }
}

hipError_t launch_score_wunits(const QueryParams &p, const uint4 *units, uint32_t n_units, uint32_t *unit_ctr, int grid,
                               hipStream_t s) {
  hipLaunchKernelGGL(k_score_wunits, dim3(grid), dim3(kWunitWaves * 64), 0, s, p, units, n_units, unit_ctr);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// All hits in (score desc, doc asc) order = searcher.search(q, Integer.MAX_VALUE)
// (Worker.java:230).  k_score_blocks leaves one sorted run per doc block
// (hits[b * kBlockDocs ...], hits_n[b] keys); k_hits_prefix turns the run
// lengths into output offsets P[0..R]; k_merge_runs merges pairs of runs
// level by level (merge path: each thread co-ranks the start of its kMergeOut-output
// chunk by binary search, then merges sequentially).  Keys are unique, so the
// result is the deterministic descending key order.  The last level writes
// (doc, score) split, or packed keys with a caller doc base (multi-GPU).
__global__ void __launch_bounds__(1024) k_hits_prefix(const uint32_t *hits_n, uint32_t R, uint64_t *P) {
  __shared__ uint64_t wsum[16];
  __shared__ uint64_t carry;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < R; base += 1024) {
    const uint32_t i = base + tid;
    const uint64_t v = i < R ? hits_n[i] : 0u;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(x, o, 64);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint64_t pre = carry;
    for (uint32_t w = 0; w < wv; w++) pre += wsum[w];
    if (i < R) P[i] = pre + x - v;
    __syncthreads();
    if (tid == 1023) carry = pre + x;
    __syncthreads();
  }
  if (tid == 0) P[R] = carry;
}

struct MergeRunsParams {
  const uint64_t *src;
  uint64_t *dst;            // packed keys out (non-final levels, or final with keys_out)
  const uint64_t *P;        // [R + 1] output offsets of the block runs
  uint32_t R, level;
  uint32_t gapped;          // level 0: run r starts at src + r * kBlockDocs
  uint32_t final;           // last level: write out_doc / out_score (or keys with doc_base into dst)
  uint32_t *out_doc;
  float *out_score;
  uint64_t doc_base;
};

#ifndef TFIDF_MERGE_OUT
#define TFIDF_MERGE_OUT 2
#endif
// outputs per thread: a co-rank search, then a sequential merge whose loads depend on
// each other; 8 -> 2 cut the all-hits device time 0.096 -> 0.079 ms (1 measured the same)
constexpr uint32_t kMergeOut = TFIDF_MERGE_OUT;
__global__ void __launch_bounds__(256) k_merge_runs(MergeRunsParams p) {
  const uint64_t H = p.P[p.R];
  const uint32_t span = 1u << (p.level + 1), half = 1u << p.level;
  const uint32_t npairs = (p.R + span - 1) / span;
  const uint64_t nchunks = (H + kMergeOut - 1) / kMergeOut;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t o = c * kMergeOut;
    const uint64_t oend = min(o + kMergeOut, H);
    while (o < oend) {
      // pair holding output o: the last pair whose first offset is <= o
      uint32_t lo = 0, hi = npairs - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (p.P[min((uint64_t)mid * span, (uint64_t)p.R)] <= o) lo = mid; else hi = mid - 1;
      }
      const uint32_t a0 = lo * span, a1 = min(a0 + half, p.R), b1 = min(a0 + span, p.R);
      const uint64_t ps = p.P[a0], pm = p.P[a1], pe = p.P[b1];
      const uint64_t la = pm - ps, lb = pe - pm;
      const uint64_t *A = p.src + (p.gapped ? (uint64_t)a0 * kBlockDocs : ps);
      const uint64_t *Bv = p.src + (p.gapped ? (uint64_t)a1 * kBlockDocs : pm);
      // co-rank: ia = outputs of [ps, o) taken from A
      const uint64_t j = o - ps;
      uint64_t ia_lo = j > lb ? j - lb : 0, ia_hi = min(j, la);
      while (ia_lo < ia_hi) {
        const uint64_t mid = (ia_lo + ia_hi) >> 1;
        if (A[mid] > Bv[j - mid - 1]) ia_lo = mid + 1; else ia_hi = mid;
      }
      uint64_t ia = ia_lo, ib = j - ia_lo;
      const uint64_t stop = min(oend, pe);
      for (; o < stop; o++) {
        uint64_t key;
        if (ib >= lb || (ia < la && A[ia] > Bv[ib])) key = A[ia++];
        else key = Bv[ib++];
        if (!p.final) {
          p.dst[o] = key;
        } else {
          const uint32_t doc = ~(uint32_t)(key & 0xFFFFFFFFull);
          if (p.out_doc) {
            p.out_doc[o] = doc;
            p.out_score[o] = __uint_as_float((uint32_t)(key >> 32));
          } else {
            p.dst[o] = (key & 0xFFFFFFFF00000000ull) | (uint64_t)(~(uint32_t)(doc + p.doc_base));
          }
        }
      }
    }
  }
}

// Levels 0-2 in one launch: workgroup g merges runs [8g, 8g + 8) (an 8-way
// merge as three pairwise levels).  A group of <= kGroupCap keys is staged in
// LDS once (ping-pong halves), merged there level by level, and written out
// compact at its output offset; a larger group runs the same three levels
// through global memory (spare, dst) inside the workgroup.  The remaining
// levels (3, 4, ...) are k_merge_runs over the compact group runs.
constexpr uint32_t kGroupRuns = 8;
constexpr uint32_t kGroupCap = 8192;
constexpr uint32_t kGroupThreads = 1024;

// merge outputs [o, oend) of one level of a group: runs start at rb[] (compact
// offsets, rb[kGroupRuns] = n), pairs of span runs
__device__ __forceinline__ void group_level_chunk(const uint64_t *S, uint64_t *D, const uint32_t *rb, uint32_t span,
                                                  uint32_t o, uint32_t oend) {
  const uint32_t half = span >> 1;
  while (o < oend) {
    uint32_t m = 0;                                             // pair holding output o
    for (uint32_t c = span; c < kGroupRuns; c += span)
      if (rb[c] <= o) m = c;
    const uint32_t ps = rb[m], pm = rb[min(m + half, kGroupRuns)], pe = rb[min(m + span, kGroupRuns)];
    const uint32_t la = pm - ps, lb = pe - pm;
    const uint64_t *A = S + ps, *Bv = S + pm;
    const uint32_t j = o - ps;
    uint32_t lo = j > lb ? j - lb : 0, hi = min(j, la);
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (A[mid] > Bv[j - mid - 1]) lo = mid + 1; else hi = mid;
    }
    uint32_t ia = lo, ib = j - lo;
    const uint32_t stop = min(oend, pe);
    for (; o < stop; o++) {
      if (ib >= lb || (ia < la && A[ia] > Bv[ib])) D[o] = A[ia++];
      else D[o] = Bv[ib++];
    }
  }
}

__global__ void __launch_bounds__(kGroupThreads) k_merge_group(MergeRunsParams p, uint64_t *spare) {
  extern __shared__ uint64_t lds[];                             // [2][kGroupCap]
  __shared__ uint32_t rb[kGroupRuns + 1];
  const uint32_t tid = threadIdx.x;
  const uint32_t r0 = blockIdx.x * kGroupRuns;
  const uint64_t ps = p.P[r0];
  if (tid <= kGroupRuns) rb[tid] = (uint32_t)(p.P[min(r0 + tid, p.R)] - ps);
  __syncthreads();
  const uint32_t n = rb[kGroupRuns];
  if (n == 0) return;                                           // workgroup-uniform
  const bool in_lds = n <= kGroupCap;
  uint64_t *X = in_lds ? lds : spare + ps, *Y = in_lds ? lds + kGroupCap : p.dst + ps;
  // gapped runs (run r at src + r * kBlockDocs) -> compact X
  for (uint32_t i = tid; i < n; i += kGroupThreads) {
    uint32_t r = 0;
#pragma unroll
    for (uint32_t c = 1; c < kGroupRuns; c++) r = rb[c] <= i ? c : r;
    X[i] = p.src[(uint64_t)(r0 + r) * kBlockDocs + (i - rb[r])];
  }
  __syncthreads();
  const uint32_t per = (n + kGroupThreads - 1) / kGroupThreads;
  for (uint32_t span = 2; span <= kGroupRuns; span <<= 1) {      // X -> Y, swap
    const uint32_t o = min(tid * per, n), oend = min(o + per, n);
    group_level_chunk(X, Y, rb, span, o, oend);
    __syncthreads();
    uint64_t *t = X; X = Y; Y = t;
  }
  // X holds the merged group (global path: spare, dst, spare, dst -> dst after 3 levels)
  for (uint32_t i = tid; i < n; i += kGroupThreads) {
    const uint64_t key = X[i], o = ps + i;
    if (!p.final) {
      if (in_lds) p.dst[o] = key;                               // (global path: already in dst)
    } else {
      const uint32_t doc = ~(uint32_t)(key & 0xFFFFFFFFull);
      if (p.out_doc) {
        p.out_doc[o] = doc;
        p.out_score[o] = __uint_as_float((uint32_t)(key >> 32));
      } else {
        p.dst[o] = (key & 0xFFFFFFFF00000000ull) | (uint64_t)(~(uint32_t)(doc + p.doc_base));
      }
    }
  }
}

hipError_t launch_hits_order(const uint64_t *hits, const uint32_t *hits_n, uint32_t R, uint64_t *P, uint64_t *tmp0,
                             uint64_t *tmp1, uint64_t *tmp2, uint32_t *out_doc, float *out_score, uint64_t *keys_out,
                             uint64_t doc_base, uint64_t hits_bound, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_hits_prefix, dim3(1), dim3(1024), 0, s, hits_n, R, P);
  uint32_t levels = 1;
  while ((1u << levels) < R) levels++;
  MergeRunsParams mp{};
  mp.P = P;
  mp.R = R;
  mp.doc_base = doc_base;
  const uint64_t *src = hits;
  uint64_t *bufs[2] = {tmp0, tmp1};
  uint32_t L0 = 0;
  // Group merging pays when the groups fit in LDS: used when the query's hit
  // bound (sum of its scoring terms' df) averages <= kHitsGroupAvg per group; a
  // group that overflows anyway is merged correctly, one workgroup through
  // global memory (slow: k_merge_group 22 us on average with the bench's heavy
  // queries included).  TFIDF_HITS_PAIRWISE / TFIDF_HITS_GROUPS force a path (tests).
  bool groups = hits_bound * kGroupRuns <= (uint64_t)R * kHitsGroupAvg;
  if (knob("TFIDF_HITS_PAIRWISE")) groups = false;
  if (knob("TFIDF_HITS_GROUPS")) groups = true;
  if (groups) {                                                 // levels 0-2: one workgroup per 8 runs
    static std::atomic<uint64_t> big{0};
    allow_dyn_lds((const void *)k_merge_group, 2 * kGroupCap * 8, big);
    mp.src = hits;
    mp.gapped = 1;
    mp.final = levels <= 3;
    mp.dst = mp.final && keys_out ? keys_out : tmp0;
    mp.out_doc = mp.final && !keys_out ? out_doc : nullptr;
    mp.out_score = mp.final && !keys_out ? out_score : nullptr;
    hipLaunchKernelGGL(k_merge_group, dim3((R + kGroupRuns - 1) / kGroupRuns), dim3(kGroupThreads),
                       2 * kGroupCap * 8, s, mp, tmp2);
    if (mp.final) return hipGetLastError();
    src = tmp0;                                                 // level 2's buffer (bufs[0])
    L0 = 3;
  }
  for (uint32_t L = L0; L < levels; L++) {
    mp.src = src;
    mp.level = L;
    mp.gapped = L == 0;
    mp.final = L + 1 == levels;
    mp.dst = mp.final && keys_out ? keys_out : bufs[L & 1];
    mp.out_doc = mp.final && !keys_out ? out_doc : nullptr;
    mp.out_score = mp.final && !keys_out ? out_score : nullptr;
    hipLaunchKernelGGL(k_merge_runs, dim3(grid), dim3(256), 0, s, mp);
    src = bufs[L & 1];
  }
  return hipGetLastError();
}

// top-k results of n_q queries -> packed merge keys with a doc base (the
// multi-GPU all-gather form: score bits << 32 | ~global doc; 0 = empty slot)
__global__ void k_pack_keys(const uint32_t *out_doc, const float *out_score, const uint32_t *out_n, uint32_t n_q,
                            uint32_t k, uint64_t doc_base, uint64_t *keys) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)n_q * k) return;
  const uint32_t q = (uint32_t)(i / k), j = (uint32_t)(i - (uint64_t)q * k);
  keys[i] = j < out_n[q] ? ((uint64_t)__float_as_uint(out_score[i]) << 32) |
                               (uint64_t)(~(uint32_t)(out_doc[i] + doc_base))
                         : 0ull;
}

hipError_t launch_pack_keys(const uint32_t *out_doc, const float *out_score, const uint32_t *out_n, uint32_t n_q,
                            uint32_t k, uint64_t doc_base, uint64_t *keys, hipStream_t s) {
  const uint64_t n = (uint64_t)n_q * k;
  if (n) hipLaunchKernelGGL(k_pack_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, out_doc, out_score, out_n, n_q,
                            k, doc_base, keys);
  return hipGetLastError();
}

hipError_t launch_score_pairs(const QueryParams &p, int grid, hipStream_t s) {
  if (p.toff) hipLaunchKernelGGL(k_score_pairs<true>, dim3(grid), dim3(kPairWaves * 64), 0, s, p);
  else hipLaunchKernelGGL(k_score_pairs<false>, dim3(grid), dim3(kPairWaves * 64), 0, s, p);
  return hipGetLastError();
}

template <bool kTerm>
static void score_blocks_layout(const QueryParams &p, dim3 grid, hipStream_t s) {
  if (p.k == 0) {
    if (p.ops) hipLaunchKernelGGL((k_score_blocks<true, true, kTerm>), grid, dim3(kScoreThreads), 0, s, p);
    else hipLaunchKernelGGL((k_score_blocks<false, true, kTerm>), grid, dim3(kScoreThreads), 0, s, p);
  } else {
    if (p.ops) hipLaunchKernelGGL((k_score_blocks<true, false, kTerm>), grid, dim3(kScoreThreads), 0, s, p);
    else hipLaunchKernelGGL((k_score_blocks<false, false, kTerm>), grid, dim3(kScoreThreads), 0, s, p);
  }
}

hipError_t launch_score_blocks(const QueryParams &p, hipStream_t s) {
  const dim3 grid = p.ovf_list ? dim3(p.list_grid) : dim3(p.n_blocks, (p.n_q + p.q_chunk - 1) / p.q_chunk);
  if (p.toff) score_blocks_layout<true>(p, grid, s);
  else score_blocks_layout<false>(p, grid, s);
  return hipGetLastError();
}
// Wave per query: the same merge for up to kMergeWaveRegs x 64 candidate slots
// (n_blocks x k; cfg 2: 123 x 10) and k <= 64, all in registers — no
// workgroup barriers (k_merge_topk's 1024-thread radix passes: 17 us for one
// query).  Keys are unique: radix select of the k-th largest from the first
// differing bit (8-bit digits, wave histogram in LDS, wave_select_bin), then
// the winners are gathered one per lane and bitonic-sorted (descending).

__global__ void __launch_bounds__(64 * kMergeWavesPerWG) k_merge_topk_wave(QueryParams p) {
  __shared__ uint32_t hist_all[kMergeWavesPerWG][256];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t q = blockIdx.x * kMergeWavesPerWG + w;
  uint32_t *hist = hist_all[w];
  for (uint32_t i = lane; i < 256; i += 64) hist[i] = 0;
  if (q >= p.n_q) return;                                   // wave-uniform; the wave owns its histogram
  merge_query_wave(p, q, hist);
}

hipError_t launch_merge_topk(const QueryParams &p, hipStream_t s) {
  if (p.k <= 64 && (uint64_t)p.n_blocks * p.k <= 64u * kMergeWaveRegs && !knob("TFIDF_MERGE_WG"))
    hipLaunchKernelGGL(k_merge_topk_wave, dim3((p.n_q + kMergeWavesPerWG - 1) / kMergeWavesPerWG),
                       dim3(64 * kMergeWavesPerWG), 0, s, p);
  else
    hipLaunchKernelGGL(k_merge_topk, dim3(p.n_q), dim3(1024), 0, s, p);
  return hipGetLastError();
}

}  // namespace tfidf
