// tfidf_internal.h — kernel parameter blocks and launch wrappers (host side).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>

#include "tfidf_common.h"

namespace tfidf {

// Debug, test and A/B knobs (TFIDF_* environment variables other than
// TFIDF_DEBUG): read only while TFIDF_DEBUG is set, so a stray variable in a
// host process's environment (a JVM inherits its parent's) never changes the
// kernel path of the library.  Without TFIDF_DEBUG every knob is unset.
inline const char *knob(const char *name) {
  const char *d = getenv("TFIDF_DEBUG");
  if (!d || !*d || (d[0] == '0' && !d[1])) return nullptr;
  return getenv(name);
}

// Error flags raised by kernels (device word err[0]; err[1] = first doc).
constexpr uint32_t kErrCapacity = 4u;
constexpr uint32_t kErrTfTooLarge = 8u;
constexpr uint32_t kErrLongScratch = 16u;
constexpr uint32_t kErrCollision = 32u;   // two different terms under one hashed key: rebuild with another seed

// Long-document path: chunks of kChunk bytes, global per-document table.
constexpr uint32_t kChunk = 2048;
constexpr uint32_t kPreMargin = 64;
constexpr uint32_t kPostMargin = 320;
constexpr uint64_t kLongScratchBudget = 8ull << 30;   // per-document tables of the concurrent long-path workgroups

struct BuildParams {
  const uint8_t *text;        // corpus base (device)
  const uint64_t *offsets;    // staged doc offsets [n_staged + 1]
  const uint32_t *live_map;   // committed doc -> staged doc (nullptr = identity)
  uint64_t n_docs;            // committed docs
  uint64_t *dict;             // 3*C u64: lo[C] (key lo per slot), hi[C], ref[C] (dict_device.h)
  uint64_t hash_seed;         // KeyBuilder seed of this build (tfidf_common.h)
  uint64_t *verify_defer;     // hashed-key checks whose reference was not visible yet: (slot, ref word)
  uint32_t *verify_count;
  uint32_t verify_cap;
  uint32_t cap_mask;          // C - 1
  uint32_t range_shift;       // log2(range size)
  uint32_t n_ranges;          // R = C >> range_shift
  uint32_t *csr;              // padded CSR rows, one packed word per entry (csr_pack)
  uint64_t *csr_esc;          // escape list: (entry index << 24) | tf for tfs the packed field cannot hold
  uint32_t *esc_count;
  uint64_t esc_cap;
  uint32_t *doc_len;          // tokens per doc (field length)
  uint32_t *doc_nuniq;        // distinct terms per doc
  uint8_t *doc_norm;          // SmallFloat.intToByte4(len)
  uint32_t *rsplit;           // [n_docs][R] inclusive end of each range segment in the row
  uint32_t *long_list;        // docs deferred to the long path
  uint32_t *long_count;
  uint32_t *uni_list;         // per document: 1 = the ASCII wave path found non-ASCII bytes (Unicode wave path)
  uint32_t *uni_count;        // flagged documents
  uint32_t *uni_wave_count;   // flagged documents k_tokenize_wave<UNI> took (the rest: k_tokenize_uwave)
  uint32_t *bad_list;         // docs that are not valid UTF-8 (indexed empty; tfidf_malformed_docs)
  uint32_t *bad_count;
  unsigned long long *stats;  // [0] docCount, [1] sumTotalTermFreq, [2] nnz
  uint32_t *err;              // [0] flags, [1] first offending doc
  // long path scratch (one table region per workgroup)
  uint64_t *lt_keys;          // 2 * lt_slots per workgroup
  uint64_t *lt_pos;           // lt_slots per workgroup: first occurrence (dict_ref_word, document-relative)
  uint32_t *lt_cnt;           // lt_slots per workgroup
  uint32_t *lt_g;             // lt_slots per workgroup
  uint32_t lt_slots_log2;     // table slots per workgroup (max)
  uint32_t debug_stop;        // profiling only (TFIDF_DEBUG_STOP): end each document after phase N
  uint32_t debug_uw_full;     // A/B only (TFIDF_UW_FULL): the Unicode wave path always scans whole documents
  // wave path units: pack > 1 = packs of `pack` consecutive documents per
  // window (short-document corpora); documents a pack cannot take go to
  // retry_list.  doc_list (pack <= 1): process these documents only
  // (*doc_list_count of them) instead of 0..n_docs-1.
  uint32_t pack;
  uint32_t *retry_list;
  uint32_t *retry_count;
  const uint32_t *doc_list;
  const uint32_t *doc_list_count;
  // book-sized documents, chunk-parallel (k_tokenize_chunk / k_long_rows):
  // the group's documents, their first unit (chunk_pre[n_group_docs + 1],
  // unit = (document, core)), each unit's pair list (kWaveTerms u32 words:
  // (slot & (2^pair_bshift - 1)) << kPairTfBits | tf, grouped by bucket
  // slot >> pair_bshift) with its pair_nb + 1 bucket starts, failure flags
  const uint32_t *chunk_pre;
  uint32_t n_group_docs;
  uint64_t n_chunks;
  const uint32_t *chunk_docs;
  uint32_t *pairs;
  uint32_t *pair_ub;
  uint32_t pair_bshift, pair_nb;
  uint32_t *chunk_fail;
  // units whose window holds non-ASCII text: k_tokenize_chunk lists them for
  // k_tokenize_uchunk (nullptr: such a unit fails its document)
  uint32_t *uchunk_list;
  uint32_t *uchunk_count;
};

__host__ __device__ inline uint64_t csr_row_base(const uint64_t *offsets, uint64_t src) {
  // A document of L bytes holds at most ceil(L/2) tokens, so rows laid out at
  // floor((offset + src) / 2) never overlap.
  return (offsets[src] + src) >> 1;
}

// Packed CSR entry, one u32 per (document, distinct term): bits [0,
// range_shift) = the term's dictionary slot minus its range base (the row
// segment it sits in names the range, rsplit), bits [range_shift, 32) = tf.
// A tf the field cannot hold stores the all-ones escape there and the exact
// value goes to the escape list ((entry index << 24) | tf, sorted by the host
// after the build, binary-searched).  Block-major ranges are 2^15 slots, so
// the field is 17 bits and only book-sized documents can escape; term-major
// rows keep the whole slot (range_shift = log2 C).  A word is never 0 (tf >= 1).
__host__ __device__ inline uint32_t csr_esc_value(uint32_t range_shift) { return 0xFFFFFFFFu >> range_shift; }
__host__ __device__ inline uint32_t csr_local(uint32_t e, uint32_t range_shift) {
  return e & ((1u << range_shift) - 1u);
}
__host__ __device__ inline uint32_t csr_tf_field(uint32_t e, uint32_t range_shift) { return e >> range_shift; }

// tf of escaped entry idx (0 if absent)
__host__ __device__ inline uint32_t csr_esc_tf(const uint64_t *esc, uint64_t n, uint64_t idx) {
  uint64_t a = 0, z = n;
  while (a < z) {
    const uint64_t m = (a + z) >> 1;
    if ((esc[m] >> 24) < idx) a = m + 1; else z = m;
  }
  return a < n && (esc[a] >> 24) == idx ? (uint32_t)(esc[a] & 0xFFFFFFu) : 0u;
}

}  // namespace tfidf
#if defined(__HIPCC__)
#include "dict_device.h"
#include "unicode_scan.h"
#endif
namespace tfidf {
#if defined(__HIPCC__)
// Cold parameters of the BuildParams kernels (every one takes the block as its
// only argument, so it sits at offset 0 of the kernarg segment): read at the
// point of use.  The asm makes the pointer opaque, so the scalar load is not
// hoisted out of the document loop and its value not kept live in SGPRs (the
// wave tokenizer used to spill ~100 of them to VGPR lanes and restore them
// with v_readlane in its hot loops).
typedef const BuildParams __attribute__((address_space(4))) KBuildParams;
__device__ __forceinline__ KBuildParams *cold_args() {
  KBuildParams *q = (KBuildParams *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return q;
}
#define TFIDF_COLD(f) (cold_args()->f)

__device__ inline void set_build_err(uint32_t *err, uint32_t flag, uint32_t doc) {
  const uint32_t old = atomicOr(err, flag);
  if (old == 0) atomicExch(err + 1, doc);
}
// Exact identity of a hashed term that resolved to global dictionary slot
// `slot` without claiming it: its occurrence `mine` (dict_ref_word) must
// spell the same term as the slot's reference occurrence.  A reference not
// visible yet (claimed by another wave just now) defers the check to
// k_verify_deferred after the tokenizers.
__device__ inline void dict_verify(const BuildParams &p, uint32_t slot, uint64_t mine, uint32_t doc) {
  const uint64_t r = __hip_atomic_load(p.dict + 2 * ((size_t)p.cap_mask + 1) + slot, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  if (r == mine) return;
  if (r == 0) {
    const uint32_t at = atomicAdd(TFIDF_COLD(verify_count), 1u);
    if (at < TFIDF_COLD(verify_cap)) {
      uint64_t *vd = TFIDF_COLD(verify_defer);
      vd[2 * (size_t)at] = slot;
      vd[2 * (size_t)at + 1] = mine;
    } else {
      set_build_err(TFIDF_COLD(err), kErrCollision, doc);   // cannot defer: treated as a collision (rebuild)
    }
    return;
  }
  if (!uc_same_term(p.text + dict_ref_off(r), dict_ref_len(r), p.text + dict_ref_off(mine), dict_ref_len(mine)))
    set_build_err(TFIDF_COLD(err), kErrCollision, doc);
}

// write CSR entry idx of document doc (dictionary slot, tf)
__device__ inline void csr_put(const BuildParams &p, uint64_t idx, uint32_t slot, uint32_t tf, uint32_t doc) {
  const uint32_t esc = csr_esc_value(p.range_shift);
  uint32_t f = tf;
  if (tf >= esc) {
    f = esc;
    if (tf > kMaxTf) set_build_err(TFIDF_COLD(err), kErrTfTooLarge, doc);
    const uint32_t at = atomicAdd(TFIDF_COLD(esc_count), 1u);
    if (at < TFIDF_COLD(esc_cap)) TFIDF_COLD(csr_esc)[at] = (idx << 24) | (tf > kMaxTf ? kMaxTf : tf);
  }
  __builtin_nontemporal_store(csr_local(slot, p.range_shift) | (f << p.range_shift), p.csr + idx);   // read by the next kernel
}
#endif

// Block-major posting (one u32): document within its 8192-doc block (13
// bits) | min(tf, kPostTfEsc) << 13 | norm byte << 24.  tf >= kPostTfEsc
// (2047 occurrences of a term in one document) is an escape: the exact value
// is in the sorted posting escape list (csr_esc_tf format, keyed by posting
// index).  Term-major postings stay u64: doc | (tf << 8 | norm) << 32.
constexpr uint32_t kPostTfEsc = 2047;
__host__ __device__ inline uint32_t post_word(uint32_t doc_local, uint32_t tf, uint32_t norm) {
  return doc_local | ((tf < kPostTfEsc ? tf : kPostTfEsc) << 13) | (norm << 24);
}

struct PostingParams {
  const uint64_t *offsets;
  const uint32_t *live_map;
  uint64_t n_docs;
  uint32_t C;                 // dictionary slots
  uint32_t range_shift, n_ranges;
  uint32_t n_blocks;          // ceil(n_docs / kBlockDocs)
  const uint32_t *csr, *rsplit;
  const uint64_t *csr_esc;    // sorted escape list (csr_put)
  uint64_t n_esc;
  const uint8_t *doc_norm;
  uint32_t NC;                // columns: occupied dictionary slots (block-major: num_terms)
  const uint2 *crank;         // [C / 32 + 1] {occupancy bits, occupied slots before} per 32 slots (col_rank)
  uint32_t *blk;              // [(n_blocks + 1) * NC]: per-block term counts -> per-block exclusive
                              // offsets over columns; row n_blocks = df per column
  uint64_t *bbase;            // [n_blocks + 1]: first posting of each block (block-major postings)
  uint32_t *post;             // [nnz] block-major postings (post_word); block b, column c at
                              // bbase[b] + blk[b][c]
  uint64_t *post_esc;         // (posting index << 24) | tf for tf >= kPostTfEsc
  uint32_t *post_esc_count;
  uint64_t post_esc_cap;
  uint32_t *err;
  uint32_t *post_tmp;         // [nnz] scatter pass 1 output (sub-range streams, same regions)
  uint32_t sort_spw;          // scatter pass 2: sub-range streams per workgroup
};

// Raise a kernel's dynamic-LDS limit on the current device, once per device:
// the attribute applies to the device current at the call, so a process with
// indices on several GPUs sets it on each (idempotent, so concurrent first
// calls are harmless).
inline void allow_dyn_lds(const void *fn, int bytes, std::atomic<uint64_t> &done_mask) {
  int dev = 0;
  hipGetDevice(&dev);
  const uint64_t bit = 1ull << (dev & 63);
  if (done_mask.load(std::memory_order_acquire) & bit) return;
  hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  done_mask.fetch_or(bit, std::memory_order_acq_rel);
}

// --- launch wrappers (kernels_index.hip) ---
hipError_t launch_tokenize_wave(const BuildParams &p, int grid, hipStream_t s);
hipError_t launch_tokenize_wave_uni(const BuildParams &p, int grid, hipStream_t s);   // flagged non-ASCII documents
hipError_t launch_tokenize_chunks_uni(const BuildParams &p, int grid, hipStream_t s);  // flagged non-ASCII book units
constexpr uint32_t kWaveWGsPerCU = 8;       // 64-thread workgroups per CU (2 waves/SIMD: VGPR- and LDS-bound)
constexpr uint32_t kWaveGroups = 128;     // CSR row groups per wave unit (documents x ranges, k_tokenize_wave)
constexpr uint32_t kPackMaxDocs = 16;     // documents per packed window (<= kPackMax, kernels_index.hip)
constexpr uint64_t kPackBytes = 2560;     // text per packed window (auto pack size): ~450 tokens, under the
                                          // wave table's 512 distinct terms (cfg 5: 7 docs, tokenize 16.3 -> 14.9 ms)
hipError_t launch_tokenize_long(const BuildParams &p, int grid, hipStream_t s);
constexpr uint32_t kLongCoreBytes = 2048;              // = kCoreBytes (kernels_index.hip)
constexpr uint64_t kPairBudget = 2ull << 30;           // per-group unit pair lists (book-sized documents)
constexpr uint32_t kPairWords = 512;                    // pair list capacity per unit (= kWaveTerms)
#ifndef TFIDF_LR_WIN_BITS
#define TFIDF_LR_WIN_BITS 15
#define TFIDF_LR_THREADS 1024
#endif
#ifndef TFIDF_LR_IN
#define TFIDF_LR_IN 16
#define TFIDF_LR_UPT 2
#endif
#ifdef TFIDF_LR_WPE
#define TFIDF_LR_ATTR __attribute__((amdgpu_waves_per_eu(TFIDF_LR_WPE)))
#else
#define TFIDF_LR_ATTR
#endif
constexpr uint32_t kLrWinBits = TFIDF_LR_WIN_BITS;      // k_long_rows: LDS window of 2^kLrWinBits u32 counters (<= a range)
constexpr uint32_t kLrWin = 1u << kLrWinBits;
constexpr uint32_t kLrThreads = TFIDF_LR_THREADS;       // k_long_rows workgroup (kLrWin / kLrThreads <= 32)
static_assert(kLrWinBits <= kRangeBits && kLrWin / kLrThreads <= 32 && kLrWin / kLrThreads >= 4, "k_long_rows window");
constexpr uint32_t kPairTfBits = 12;                    // tf field of a pair word (a 2 KB core holds < 2^11 tokens)
hipError_t launch_tokenize_chunks(const BuildParams &p, int grid, hipStream_t s);
hipError_t launch_long_rows(const BuildParams &p, uint32_t n_docs, hipStream_t s);
hipError_t launch_tokenize_uwave(const BuildParams &p, int grid, hipStream_t s);   // kernels_unicode.hip
hipError_t launch_tokenize_uchunk(const BuildParams &p, int grid, hipStream_t s);  // kernels_unicode.hip
constexpr uint32_t kUwaveWGsPerCU = 7;    // 64-thread workgroups, ~22 KB LDS each (two waves per SIMD)
constexpr uint32_t kUchunkWGsPerCU = 8;   // k_tokenize_uchunk: ~19 KB LDS each
hipError_t launch_verify_deferred(const BuildParams &p, hipStream_t s);           // kernels_index.hip
hipError_t launch_df_partial(const PostingParams &p, hipStream_t s);
hipError_t launch_df_sum(const PostingParams &p, hipStream_t s);
hipError_t launch_row_scan(const PostingParams &p, hipStream_t s);
hipError_t launch_block_base(const PostingParams &p, hipStream_t s);
hipError_t launch_count_nonzero(const uint64_t *a, uint32_t n, unsigned long long *out, hipStream_t s);
// block-major columns: crank over the final dictionary (total -> *n_cols), per-slot df from the column df
hipError_t launch_col_rank(const uint64_t *dict_lo, uint32_t C, uint2 *crank, unsigned long long *n_cols, hipStream_t s);
hipError_t launch_df_slots(const uint2 *crank, const uint32_t *df_col, uint32_t C, uint32_t *df_slot, hipStream_t s);
hipError_t launch_scatter(const PostingParams &p, hipStream_t s);

// --- term-major inversion for large vocabularies (kernels_term.hip) ---
// (hand-written LSD radix sort of packed words slot | doc | tf | norm)
constexpr uint64_t kTermMaxDocs = 1ull << 26;   // documents per shard in the term-major layout
struct TermParams {
  const uint64_t *offsets;
  const uint32_t *live_map;
  uint64_t n_docs, nnz;
  uint32_t C, slot_bits;      // C = 2^slot_bits
  uint32_t doc_bits, tf_bits; // packed word layout (kernels_term.hip TermLayout)
  const uint32_t *csr, *doc_nuniq;
  const uint64_t *csr_esc;
  uint64_t n_esc;
  const uint8_t *doc_norm;
  uint32_t *row_off;          // [n_docs] compact row offsets (exclusive sum of doc_nuniq)
  uint64_t *keys, *keys_alt;  // [nnz] each: packed words (ping-pong)
  uint64_t *tesc;             // tf >= 4095: (slot << 26 | doc, tf) u64 pairs, sorted by the host
  uint32_t *tesc_count;
  uint64_t tesc_cap, n_tesc;
  uint32_t *scratch;          // term_invert_scratch_words(n_docs, nnz) u32
  uint64_t *post;             // [nnz] out: doc | (tf << 8 | norm) << 32, term-major, docs ascending
  uint64_t *toff;             // [C + 1] out: first posting of each slot
  uint32_t *df;               // [C] out
  uint32_t *err;
};
uint64_t term_invert_scratch_words(uint64_t n_docs, uint64_t nnz, uint32_t C);
hipError_t launch_term_pairs(const TermParams &p, hipStream_t s);
hipError_t launch_term_sort(const TermParams &p, hipStream_t s);

// --- query scoring (kernels_query.hip) ---
constexpr uint32_t kInlTerms = 32;          // query terms carried in QueryParams (fused single query)
constexpr uint32_t kFusedMaxK = 64;         // tfidf_search top-k through the fused single-query launch up to this k
struct QueryParams {
  const uint64_t *post;       // term-major postings (toff != nullptr)
  const uint32_t *post32;     // block-major postings (post_word)
  const uint64_t *post_esc;   // block-major tf escapes, sorted
  uint64_t n_post_esc;
  const uint64_t *bbase;      // [n_blocks + 1] first posting of each block
  const uint32_t *blk;        // per-block exclusive offsets over columns [n_blocks * C]
  const uint64_t *toff;       // term-major layout: [C + 1] first posting per slot (nullptr = block-major)
  uint32_t C;                 // block-major: columns (num_terms); term-major: dictionary slots
  uint32_t n_blocks;
  uint64_t n_docs;
  const float *cache;         // 256 floats (BM25 norm cache)
  const uint32_t *q_off;      // [n_q + 1] into q_slot / q_w
  const uint32_t *q_slot;     // per query term: block-major column / term-major slot (kInvalidSlot = absent)
  const float *q_w;           // BM25 weight per query term (boost * idf)
  const uint32_t *q_role;     // per query term: role << 24 | MUST clause index (kRole*, tfidf_common.h)
  const uint32_t *q_meta;     // per query: MUST clause count | has MUST_NOT << 31 (0 = plain disjunction)
  uint32_t ops;               // k_score_blocks: the operator-query variant (MUST / MUST_NOT clauses)
  uint32_t n_q;
  uint32_t q_chunk;           // queries per score_blocks workgroup
  uint32_t k;                 // top-k (1..1024); 0 = all hits
  // outputs
  uint64_t *cand;             // [n_q][n_blocks][k] candidate keys (score bits << 32 | ~doc)
  uint32_t *cand_n;           // [n_q][n_blocks]
  uint32_t *out_doc;          // [n_q][k]
  float *out_score;           // [n_q][k]
  uint32_t *out_n;            // [n_q]
  // all-hits mode
  uint64_t *hits;             // [n_blocks * kBlockDocs] keys (score bits << 32 | ~doc)
  uint32_t *hits_n;           // [n_blocks]
  // wave-per-pair path (k > 0): pairs it leaves to k_score_blocks (nullptr = dense grid mode)
  uint32_t *ovf_list;         // pair ids q * n_blocks + b
  uint32_t *ovf_count;        // zeroed before k_score_pairs
  uint32_t *ovf2_list;        // pairs of operator queries (q_meta != 0), for k_score_blocks<true>
  uint32_t *ovf2_count;
  uint32_t list_grid;         // k_score_blocks workgroups in list mode
  // single query, one launch (tfidf_search, k <= 64): the query terms ride in
  // the kernel arguments (inl_n > 0: no upload) and the blocks' candidates go
  // to pinned host memory (cand / cand_n), merged by the host
  uint32_t inl_n;
  uint32_t inl_meta;
  uint32_t inl_slot[kInlTerms];
  float inl_w[kInlTerms];
  uint32_t inl_role[kInlTerms];
};
hipError_t launch_score_pairs(const QueryParams &p, int grid, hipStream_t s);
constexpr uint32_t kPairWavesPerWG = 2;   // k_score_pairs workgroup = 2 waves (30 KB LDS: 5 per CU)
hipError_t launch_score_blocks(const QueryParams &p, hipStream_t s);
// batched top-k (k <= kUnitMaxK, plain disjunctions, block-major): workgroup
// per (query, block range) unit {q, b0, b1, 0}; units of one query cover
// [0, n_blocks); unit_ctr zeroed before the launch
constexpr uint32_t kUnitMaxK = 64;
constexpr uint32_t kUnitMaxTerms = 64;
constexpr uint32_t kUnitWGsPerCU = 2;     // 71 KiB LDS each
hipError_t launch_score_units(const QueryParams &p, const uint4 *units, uint32_t n_units, uint32_t *unit_ctr, int grid,
                              hipStream_t s);
// light queries of such batches: wave per unit (hash table per block)
constexpr uint32_t kWunitWavesPerWG = kPairWavesPerWG;
constexpr uint32_t kWunitWGsPerCU = 6;    // 25 KiB LDS each (round 6: no claim list; 5 at 29 KiB before)
constexpr uint32_t kWunitLightPost = 550; // postings per block (query average) up to which a query is light (400: batch 5.80 ms, 500: 5.62, 600: 5.53, 700: 6.6 — past kWunitPassPost blocks take 16 passes;
                                          // round 5, 10 k queries at cfg 2: 450 / 500 / 550 / 600 / 650 / 700 = 5.95 / 5.94 / 5.52 / 5.53 / 5.69 / 6.53 ms device; 550 keeps a margin from the cliff)
hipError_t launch_score_wunits(const QueryParams &p, const uint4 *units, uint32_t n_units, uint32_t *unit_ctr, int grid,
                               hipStream_t s);
hipError_t launch_merge_topk(const QueryParams &p, hipStream_t s);
// all hits: per-block sorted runs (k_score_blocks, k == 0) -> one ordered list:
// (doc, score) split into out_doc / out_score, or packed keys with doc_base
// added into keys_out (when non-null).  P: R + 1 u64; tmp0 / tmp1: n_blocks *
// kBlockDocs u64 each (tmp1 may alias hits).
hipError_t launch_pack_keys(const uint32_t *out_doc, const float *out_score, const uint32_t *out_n, uint32_t n_q,
                            uint32_t k, uint64_t doc_base, uint64_t *keys, hipStream_t s);
hipError_t launch_hits_order(const uint64_t *hits, const uint32_t *hits_n, uint32_t R, uint64_t *P, uint64_t *tmp0,
                             uint64_t *tmp1, uint64_t *tmp2, uint32_t *out_doc, float *out_score, uint64_t *keys_out,
                             uint64_t doc_base, uint64_t hits_bound, int grid, hipStream_t s);
constexpr uint64_t kHitsGroupAvg = 6144;   // all hits: 8-run LDS group merge when hits per group average <= this

// --- GLOBAL statistics by term ownership (kernels_vocab.hip) ---
hipError_t vocab_count(const uint64_t *dict, uint32_t C, uint32_t G, uint32_t *counts, hipStream_t s);
hipError_t vocab_starts(const uint32_t *counts, uint32_t G, uint32_t *cursor, uint64_t *counts_out, hipStream_t s);
hipError_t vocab_scatter(const uint64_t *dict, const uint32_t *df, uint32_t C, uint32_t G, uint32_t *cursor,
                         uint64_t *records, uint32_t *sent_slot, hipStream_t s);
hipError_t vocab_reduce(const uint64_t *records, uint64_t n, uint64_t *table, uint32_t tmask, uint32_t *sums,
                        uint32_t *rslot, uint32_t *out, unsigned long long *n_unique, hipStream_t s);
hipError_t vocab_import(const uint32_t *sent_slot, const uint32_t *gdf_in, uint64_t n, uint32_t *gdf, hipStream_t s);

// --- index internals the node-level orchestration reads (tfidf_capi.hip) ---
}  // namespace tfidf
struct tfidf_index;
struct tfidf_reader;
namespace tfidf {
hipStream_t index_stream(tfidf_index *ix);
int index_device(const tfidf_index *ix);
bool index_committed(const tfidf_index *ix);
uint64_t index_num_docs(const tfidf_index *ix);
uint64_t index_generation(const tfidf_index *ix);   // successful commits so far
int set_error(int code, const char *msg);       // sets tfidf_last_error() of the calling thread
// device-key searches on a reader's pinned snapshot (tfidf_reader_open)
int reader_batch_keys_device(tfidf_reader *rd, const uint8_t *q_utf8, const uint64_t *q_offsets, uint32_t n_q,
                             uint32_t k, uint64_t doc_base, void *d_keys);
int reader_all_keys_device(tfidf_reader *rd, const uint8_t *q, uint64_t q_len, uint64_t doc_base, void *d_keys,
                           uint64_t cap, uint64_t *n_out);
// GLOBAL exchange steps without the public calls' host synchronisation (every
// buffer is the communicator's, ordered on the index's stream)
int vocab_partition_async(tfidf_index *ix, uint32_t n_ranks, void *d_records, uint64_t cap, void *d_counts,
                          uint64_t *n_out);
int vocab_reduce_async(tfidf_index *ix, const void *d_records, uint64_t n, void *d_df_out, void *d_n_unique);
int set_global_df_async(tfidf_index *ix, const void *d_df, uint64_t n, uint64_t doc_count, uint64_t sum_ttf,
                        uint64_t *generation);
// String.compareTo order of two UTF-8 names (UTF-16 code units; Leader.java:80-88 TreeMap)
int utf16_compare(const uint8_t *a, uint64_t na, const uint8_t *b, uint64_t nb);

// --- node-level merges (tfidf_dist.hip) ---
// lists (q, r) of `len` merge keys at keys + r * rstride + q * qstride, each
// sorted descending (0 = empty, last): out[q * k_out + i] = the i-th largest
// key of query q over all n_lists lists (i < k_out), 0 past the last one
hipError_t launch_merge_lists(const uint64_t *keys, uint32_t n_lists, uint64_t rstride, uint64_t qstride, uint64_t len,
                              uint32_t n_q, uint64_t *out, uint64_t k_out, hipStream_t s);

// --- synthetic corpus (kernels_synth.hip) ---
hipError_t synth_doc_lengths(uint64_t seed, uint64_t n_docs, uint64_t doc_base, const double *cdf,
                             const uint32_t *guide, uint32_t V, uint32_t len_min, uint32_t len_max,
                             uint64_t *bytes_out, hipStream_t s);
hipError_t synth_doc_text(uint64_t seed, uint64_t n_docs, uint64_t doc_base, const double *cdf,
                          const uint32_t *guide, uint32_t V, uint32_t len_min, uint32_t len_max,
                          const uint64_t *offsets, uint8_t *text, hipStream_t s);
hipError_t exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s);

#if defined(__HIPCC__)
// Book-sized documents: unit = (document, kCoreBytes core) with context
// margins (k_tokenize_chunk, k_tokenize_uchunk).
constexpr uint32_t kCoreBytes = kLongCoreBytes;
constexpr uint32_t kPreBytes = 64;
constexpr uint32_t kPostBytes = 320;
static_assert(kPreBytes + kCoreBytes + kPostBytes + 16 <= 4096, "chunk window: a wave window holds it");

struct ChunkMeta {
  uint64_t s0, L;                 // window: corpus bytes [s0, s0 + L)
  uint32_t shift, core_lo, core_hi, gi;
  uint64_t d;
};

__device__ __forceinline__ ChunkMeta chunk_meta(const BuildParams &p, uint64_t u) {
  // group document holding unit u: chunk_pre[gi] <= u < chunk_pre[gi + 1] (binary search, scalar loads)
  uint32_t lo = 0, hi = p.n_group_docs;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (p.chunk_pre[mid] <= u) lo = mid; else hi = mid;
  }
  const uint2 e = make_uint2(lo, (uint32_t)(u - p.chunk_pre[lo]));
  ChunkMeta m;
  m.gi = e.x;
  m.d = p.chunk_docs[e.x];
  const uint64_t src = p.live_map ? p.live_map[m.d] : m.d;
  const uint64_t dlo = p.offsets[src], dl = p.offsets[src + 1] - dlo;
  const uint64_t clo = (uint64_t)e.y * kCoreBytes, chi = min(dl, clo + kCoreBytes);
  const uint64_t ws = clo > kPreBytes ? clo - kPreBytes : 0, we = min(dl, chi + kPostBytes);
  m.s0 = dlo + ws;
  m.L = we - ws;
  m.core_lo = (uint32_t)(clo - ws);
  m.core_hi = (uint32_t)(chi - ws);
  m.shift = (uint32_t)(reinterpret_cast<uintptr_t>(p.text + m.s0) & 15);
  return m;
}


#endif

}  // namespace tfidf
