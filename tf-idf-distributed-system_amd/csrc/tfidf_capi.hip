// tfidf_capi.hip — the C ABI (include/tfidf.h): index lifetime, corpus
// staging, commit orchestration, query analysis and result materialisation.
// All hot-path arithmetic runs in the kernels of kernels_*.hip; this file is
// the host runtime around them (memory, streams, events, error mapping).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/tfidf.h"
#include "analysis.h"
#include "tfidf_common.h"
#include "tfidf_internal.h"

namespace tfidf {
hipError_t add_u64(uint64_t *v, uint64_t n, uint64_t delta, hipStream_t s);
hipError_t sort_unique_keys128(const uint64_t *keys, uint64_t n, uint64_t *out, uint64_t *n_unique, hipStream_t s);
hipError_t slot_to_canon(const uint64_t *dict, uint32_t C, const uint64_t *canon, uint64_t n_canon,
                         uint32_t *canon_of_slot, hipStream_t s);
hipError_t scatter_df_canon(const uint32_t *df, const uint32_t *canon_of_slot, uint32_t C, uint32_t *out,
                            hipStream_t s);
hipError_t gather_df_canon(const uint32_t *dfc, const uint32_t *canon_of_slot, uint32_t C, uint32_t *gdf,
                           hipStream_t s);
}  // namespace tfidf

using namespace tfidf;

// ---------------------------------------------------------------------------
// errors

static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                                \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    if (_e != hipSuccess) return fail(TFIDF_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                      __FILE__, __LINE__);                                           \
  } while (0)

// ---------------------------------------------------------------------------
// device buffers

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  hipError_t reserve(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    if (p) { hipFree(p); p = nullptr; bytes = 0; }
    if (n == 0) n = 16;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// pinned host array: the per-commit dictionary / df mirrors are copied at
// DMA rate instead of through pageable staging (4 MB at 2^18 slots, 128 MB at 2^23)
template <class T> struct PinnedVec {
  T *p = nullptr;
  size_t n = 0, cap = 0;
  PinnedVec() = default;
  PinnedVec(const PinnedVec &) = delete;
  PinnedVec &operator=(const PinnedVec &) = delete;
  ~PinnedVec() { if (p) hipHostFree(p); }
  hipError_t resize(size_t m) {
    if (m > cap) {
      if (p) hipHostFree(p);
      p = nullptr;
      cap = n = 0;
      hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&p), m * sizeof(T), hipHostMallocDefault);
      if (e != hipSuccess) { p = nullptr; return e; }
      cap = m;
    }
    n = m;
    return hipSuccess;
  }
  void clear() { n = 0; }
  hipError_t assign(size_t m, T v) {
    hipError_t e = resize(m);
    if (e == hipSuccess) for (size_t i = 0; i < m; i++) p[i] = v;
    return e;
  }
  T *data() { return p; }
  const T *data() const { return p; }
  size_t size() const { return n; }
  T &operator[](size_t i) { return p[i]; }
  const T &operator[](size_t i) const { return p[i]; }
};

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

// block-major rows are grouped into at most 64 dictionary ranges (the long
// path's per-range counters), i.e. C <= 64 x 32768
constexpr uint32_t kMaxBlockCapLog2 = 21;

enum { EV_START, EV_TOK, EV_L0, EV_LONG, EV_D0, EV_DF, EV_BSCAN, EV_CSCAN, EV_SCAT, EV_N };
enum { QEV_0, QEV_1, QEV_2, QEV_N };   // search timing events (per search context)

constexpr size_t kCoalesceMaxDefault = 8192;   // tfidf_search_coalesced: requests per batch

// device buffer with an owner's lifetime (freed on its device)
struct DevMem : DevBuf {
  int dev = 0;
  explicit DevMem(int d) : dev(d) {}
  DevMem(const DevMem &) = delete;
  DevMem &operator=(const DevMem &) = delete;
  ~DevMem() {
    if (p) { DeviceGuard g(dev); release(); }
  }
};

// Document keys (relative paths), append-only in chunks that never change
// once a published snapshot holds them: a snapshot keeps the chunk list it was
// committed with, the builder appends to its own last chunk (or starts a new
// one when a snapshot shares it).  Staged id -> chunk by binary search.
struct KeyChunk {
  uint64_t first = 0;                // staged id of the chunk's first document
  std::string arena;
  std::vector<uint64_t> off{0};
  std::vector<uint8_t> synth;        // 1 = key is the decimal staged id
  uint64_t size() const { return synth.size(); }
};
struct KeyTable {
  std::vector<std::shared_ptr<KeyChunk>> ch;
  const KeyChunk &chunk_of(uint64_t st) const {
    size_t a = 0, z = ch.size();
    while (z - a > 1) {
      const size_t m = (a + z) / 2;
      if (ch[m]->first <= st) a = m; else z = m;
    }
    return *ch[a];
  }
  void key(uint64_t st, std::string *out) const {
    const KeyChunk &c = chunk_of(st);
    const uint64_t i = st - c.first;
    if (c.synth[i]) *out = std::to_string(st);
    else out->assign(c.arena.data() + c.off[i], c.off[i + 1] - c.off[i]);
  }
  uint64_t key_len(uint64_t st) const {
    const KeyChunk &c = chunk_of(st);
    const uint64_t i = st - c.first;
    return c.synth[i] ? std::to_string(st).size() : c.off[i + 1] - c.off[i];
  }
  // the builder's chunk to append to (a new one when a snapshot shares the last)
  KeyChunk &tail(uint64_t n_staged) {
    if (ch.empty() || ch.back().use_count() > 1) {
      ch.push_back(std::make_shared<KeyChunk>());
      ch.back()->first = n_staged;
    }
    return *ch.back();
  }
  // flat copies (persistence)
  void flatten(std::string *arena, std::vector<uint64_t> *off, std::vector<uint8_t> *synth) const {
    arena->clear();
    off->assign(1, 0);
    synth->clear();
    for (const auto &c : ch) {
      for (uint64_t i = 0; i < c->size(); i++) {
        arena->append(c->arena, c->off[i], c->off[i + 1] - c->off[i]);
        off->push_back(arena->size());
      }
      synth->insert(synth->end(), c->synth.begin(), c->synth.end());
    }
  }
  // many small chunks (one per commit of a single upload): merge them into one
  void compact() {
    if (ch.size() <= 64) return;
    auto one = std::make_shared<KeyChunk>();
    flatten(&one->arena, &one->off, &one->synth);
    ch.assign(1, one);
  }
};

// Statistics in force for BM25 (the shard's own, or GLOBAL from the node-level
// exchange).  Never edited once a search can see it: the GLOBAL setters
// publish a new view.
struct StatsView {
  int dev = 0;
  bool global = false;
  uint64_t doc_count = 0, sum_ttf = 0;   // docCount / sumTotalTermFreq in force
  PinnedVec<uint32_t> gdf;               // GLOBAL df per dictionary slot (host mirror)
  hipEvent_t gdf_ev = nullptr;           // gdf copied (set asynchronously by tfidf_set_global_df_device)
  bool gdf_pending = false;
  std::mutex gdf_mu;
  DevMem cache;                          // 256-entry BM25 norm cache (device)
  PinnedVec<float> h_cache;
  explicit StatsView(int d) : dev(d), cache(d) {
    DeviceGuard g(d);
    hipEventCreateWithFlags(&gdf_ev, hipEventDisableTiming);
  }
  ~StatsView() {
    DeviceGuard g(dev);
    if (gdf_ev) {
      hipEventSynchronize(gdf_ev);
      hipEventDestroy(gdf_ev);
    }
  }
  int wait_gdf();                        // the GLOBAL df mirror, before its first use
};

// One committed index: everything a search reads.  Published by tfidf_commit
// as a refcounted snapshot and never changed afterwards (only its `stats`
// pointer is replaced, under the index's snap_mu); a search holds a reference
// for its whole run, so a commit never waits for searches and a search never
// waits for a commit (the reference opens a DirectoryReader on the last commit
// per request, Worker.java:223, while uploads commit beside it, :136-139).
// A snapshot no search holds any more is rebuilt in place by a later commit.
struct Snapshot {
  int dev = 0;
  uint64_t generation = 0;
  uint32_t cap_log2 = 18, C = 0, range_shift = 15, R = 1, n_blocks = 0;
  uint64_t n_docs = 0, text_bytes = 0;
  bool term_major = false;
  std::vector<uint32_t> live_map;      // committed -> staged (empty = identity)
  KeyTable keys;                       // document keys of the staged ids
  std::shared_ptr<DevMem> text, offsets;   // the staged corpus it was built from
  DevMem dict, csr, csr_esc, post_esc, doc_len, doc_nuniq, doc_norm, rsplit, blk, bbase, post, row_off, toff, tdf;
  // block-major columns (kernels_index.hip col_rank): occupancy bits and
  // prefix counts per 32 slots, the per-slot df, and the host copy of crank
  DevMem crank, sdf;
  PinnedVec<uint2> h_crank;
  uint32_t NC = 0;                     // block-major columns (= num_terms)
  std::vector<uint32_t> malformed;     // ascending committed ids of documents that are not UTF-8
  std::vector<uint64_t> h_esc;         // CSR tf escapes, sorted (csr_put)
  std::vector<uint64_t> h_post_esc;    // block-major posting tf escapes, sorted (post_word)
  uint64_t hash_seed = 0;
  uint32_t hash_rebuilds = 0;
  PinnedVec<uint64_t> h_dict;          // host mirrors for query analysis (pinned)
  PinnedVec<uint32_t> h_df;
  uint64_t doc_count = 0, sum_ttf = 0, nnz = 0, num_terms = 0, long_docs = 0;
  uint32_t pack_docs = 1;
  uint64_t pack_retried = 0, unicode_docs = 0, unicode_wave_docs = 0, long_chunked = 0;
  std::shared_ptr<StatsView> stats;    // replaced under tfidf_index::snap_mu
  std::unordered_map<uint32_t, std::string> term_cache;   // hashed slots' term strings (slot_term)
  std::mutex term_mu;
  explicit Snapshot(int d)
      : dev(d), dict(d), csr(d), csr_esc(d), post_esc(d), doc_len(d), doc_nuniq(d), doc_norm(d), rsplit(d), blk(d),
        bbase(d), post(d), row_off(d), toff(d), tdf(d), crank(d), sdf(d) {}
  const uint32_t *df_dev() const { return term_major ? tdf.as<uint32_t>() : sdf.as<uint32_t>(); }   // per slot
  // what the scorers index a term's postings by: its column (block-major) or
  // its dictionary slot (term-major); the scorers' C is the matching count
  uint32_t col_of(uint32_t slot) const {
    if (term_major) return slot;
    const uint2 e = h_crank[slot >> 5];
    return e.y + (uint32_t)__builtin_popcount(e.x & ((1u << (slot & 31u)) - 1u));
  }
  uint32_t qcols() const { return term_major ? C : NC; }
  uint64_t staged_of(uint64_t doc) const { return live_map.empty() ? doc : live_map[doc]; }
};

// Per-search scratch: a stream (plus a side stream for the batch kernels'
// fork), timing events and buffers.  Searches take a context from the index's
// pool, so concurrent searches never share one.
struct SearchCtx {
  int dev = 0;
  hipStream_t own = nullptr, side = nullptr;
  hipEvent_t ev[QEV_N] = {};
  hipEvent_t q_ev[2] = {nullptr, nullptr};  // fork / join of the wave-unit kernel on `side`
  hipEvent_t q_in_ev = nullptr;             // the last upload out of q_host
  bool q_in_pending = false;
  bool q_rec_start = true;                  // run_scoring records QEV_0 (false: a later chunk of a batch)
  bool q_timing = true;
  DevMem q_in, q_out, cand, cand_n, out_doc, out_score, hits, hits_n, hits_c, hits_s, hits_P, ovf;
  PinnedVec<uint32_t> q_host, q_res, q_cand_h;   // q_cand_h: fused single query's block candidates (host merge)
  std::vector<uint64_t> q_merge;
  std::vector<uint32_t> q_units;            // batch scoring units {q, b0, b1, 0} (run_scoring)
  uint32_t *res_doc = nullptr, *res_n = nullptr;
  float *res_score = nullptr;
  explicit SearchCtx(int d)
      : dev(d), q_in(d), q_out(d), cand(d), cand_n(d), out_doc(d), out_score(d), hits(d), hits_n(d), hits_c(d),
        hits_s(d), hits_P(d), ovf(d) {}
  int init() {
    DeviceGuard g(dev);
    if (hipStreamCreateWithFlags(&own, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&side, hipStreamNonBlocking) != hipSuccess)
      return fail(TFIDF_E_HIP, "hipStreamCreate failed");
    for (int i = 0; i < QEV_N; i++) hipEventCreate(&ev[i]);
    for (int i = 0; i < 2; i++) hipEventCreateWithFlags(&q_ev[i], hipEventDisableTiming);
    hipEventCreateWithFlags(&q_in_ev, hipEventDisableTiming);
    return TFIDF_OK;
  }
  ~SearchCtx() {
    DeviceGuard g(dev);
    if (own) hipStreamSynchronize(own);
    if (side) hipStreamSynchronize(side);
    for (int i = 0; i < QEV_N; i++) if (ev[i]) hipEventDestroy(ev[i]);
    for (int i = 0; i < 2; i++) if (q_ev[i]) hipEventDestroy(q_ev[i]);
    if (q_in_ev) hipEventDestroy(q_in_ev);
    if (side) hipStreamDestroy(side);
    if (own) hipStreamDestroy(own);
  }
};

struct tfidf_index {
  tfidf_config cfg;
  std::mutex mu;                     // writers: add_docs, commit, clear, load, the GLOBAL exchange
  hipStream_t stream = nullptr;      // the writers' stream (own_stream unless tfidf_set_stream)
  hipStream_t own_stream = nullptr;
  hipStream_t user_stream = nullptr; // tfidf_set_stream: searches run on it too
  hipEvent_t ev[EV_N];
  // side stream for the dictionary's host mirror: its D2H copy overlaps the inversion
  hipStream_t copy_stream = nullptr;
  hipEvent_t mir_ev[3];            // [0] dictionary final (main stream), [1] mirror copied, [2] df final
  int num_cus = 256;

  // published snapshot (searches) and the one a commit may rebuild in place
  std::mutex snap_mu;
  std::shared_ptr<Snapshot> cur, spare;
  uint64_t generation = 0;           // successful commits so far

  // search contexts (one per concurrent search)
  std::mutex ctx_mu;
  std::vector<std::unique_ptr<SearchCtx>> ctx_free;
  std::atomic<bool> q_timing{true};  // record HIP events around each search (tfidf_set_query_timing)
  std::mutex ms_mu;
  float last_ms_scoring = 0, last_ms_total = 0;

  // staged corpus (builder)
  std::shared_ptr<DevMem> text, offsets;   // offsets: u64[n_staged + 1]
  // corpus loader: two pinned host staging buffers, refilled while the other one's DMA runs
  void *stage[2] = {nullptr, nullptr};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  uint64_t text_bytes = 0, n_staged = 0;
  std::vector<uint64_t> h_offsets{0};
  KeyTable keys;
  std::vector<uint8_t> staged_live;
  std::unordered_map<std::string, uint64_t> key_to_staged;
  uint64_t n_dead = 0;

  // build scratch (the commit in progress)
  uint32_t cap_log2 = 18;
  DevBuf d_live_map;
  DevBuf long_list, uni_list, counters, post_tmp;
  DevBuf retry_list;                   // packed wave path: documents deferred to the single-document pass
  DevBuf bad_list;                     // documents that are not valid UTF-8 (indexed empty)
  uint64_t hash_seed = 0;              // KeyBuilder seed of the build (0 unless a collision was met)
  uint32_t hash_rebuilds = 0;          // builds redone for a hash collision in the last commit
  bool uni_first = false;              // the last commit's documents were mostly non-ASCII: UNI-first build
  uint32_t hash_floor = 0;             // first seed attempt of the next commit (tfidf_set_hash_attempt)
  uint32_t collision_doc = 0;          // a document of the last detected collision (diagnostics)
  // tfidf_search_coalesced: concurrent single top-k searches gathered into batches
  mutable std::mutex cq_mu;
  std::condition_variable cq_cv;
  std::vector<struct CoalesceReq *> cq;
  bool cq_leader = false;
  size_t cq_max = kCoalesceMaxDefault;  // requests per batch
  uint64_t cq_batches = 0, cq_queries = 0;
  std::atomic<uint64_t> unit_batches{0}, unit_count{0}, fused_queries{0};
  DevBuf verify_defer, lt_pos;
  DevBuf tvals, term_tmp, term_esc;     // term-major inversion: sort values, scratch, tf escapes
  DevBuf lt_keys, lt_cnt, lt_g;
  DevBuf pairs, pair_ub, chunk_list, chunk_docs, chunk_fail, uchunk;   // book-sized documents (chunk-parallel)
  PinnedVec<uint32_t> ldocs_h, pre_h;                            // their host staging
  PinnedVec<uint64_t> hctr_h;                                    // build counters read back after the tokenizers
  uint32_t lt_log2 = 0, lt_wgs = 64;   // lt_wgs: long-path workgroups always allowed
  tfidf_commit_timing timing{};

  // GLOBAL exchange (writers): canonical ids, record order -> slot, owner-side scratch
  DevBuf canon_of_slot;
  uint64_t n_canon = 0;
  DevBuf sent_slot, vcounts, vnu, vt_table, vt_sum, vt_rslot, gdf_dev;
  uint64_t n_sent = 0;
  // the statistics view a GLOBAL setter replaced, reused by the next one once
  // no search holds it (its pinned df mirror and device cache stay allocated)
  std::shared_ptr<StatsView> view_spare;
};

int StatsView::wait_gdf() {
  std::lock_guard<std::mutex> lk(gdf_mu);
  if (gdf_pending) {
    HIP_TRY(hipEventSynchronize(gdf_ev));
    gdf_pending = false;
  }
  return TFIDF_OK;
}

// the published snapshot and its statistics view (both null before the first commit)
static std::shared_ptr<Snapshot> current(tfidf_index *ix, std::shared_ptr<StatsView> *v = nullptr) {
  std::lock_guard<std::mutex> lk(ix->snap_mu);
  if (v) *v = ix->cur ? ix->cur->stats : nullptr;
  return ix->cur;
}
static std::shared_ptr<Snapshot> current(const tfidf_index *ix, std::shared_ptr<StatsView> *v = nullptr) {
  return current(const_cast<tfidf_index *>(ix), v);
}

// A search context from the pool (created on demand), returned on scope exit.
struct CtxLease {
  tfidf_index *ix;
  std::unique_ptr<SearchCtx> c;
  int rc = TFIDF_OK;
  explicit CtxLease(tfidf_index *x) : ix(x) {
    {
      std::lock_guard<std::mutex> lk(ix->ctx_mu);
      if (!ix->ctx_free.empty()) {
        c = std::move(ix->ctx_free.back());
        ix->ctx_free.pop_back();
      }
    }
    if (!c) {
      c.reset(new SearchCtx(ix->cfg.device));
      rc = c->init();
    }
    c->q_timing = ix->q_timing.load();
  }
  // A search returns its snapshot reference after its lease (declared later,
  // destroyed first): no kernel of a failed search may still read the
  // snapshot's buffers when a commit rebuilds that snapshot as its spare
  // (use_count() == 1).  Successful searches have synchronised already; an
  // error return (HIP_TRY, a failed preparation after earlier chunks were
  // queued) is drained here.
  ~CtxLease() {
    if (!c || rc) return;
    {
      DeviceGuard g(ix->cfg.device);
      const hipStream_t st = stream();
      if (hipStreamQuery(st) != hipSuccess) hipStreamSynchronize(st);
      if (c->side && hipStreamQuery(c->side) != hipSuccess) hipStreamSynchronize(c->side);
    }
    std::lock_guard<std::mutex> lk(ix->ctx_mu);
    ix->ctx_free.push_back(std::move(c));
  }
  hipStream_t stream() const { return ix->user_stream ? ix->user_stream : c->own; }
};

// ---------------------------------------------------------------------------

extern "C" const char *tfidf_version(void) { return "libtfidf 0.1.0 (gfx950)"; }
extern "C" const char *tfidf_last_error(void) { return g_err.c_str(); }

extern "C" int tfidf_config_init(tfidf_config *cfg) {
  if (!cfg) return fail(TFIDF_E_INVALID_ARG, "cfg is NULL");
  cfg->k1 = 1.2f;
  cfg->b = 0.75f;
  cfg->stats_mode = TFIDF_STATS_SHARD;
  cfg->device = 0;
  cfg->vocab_capacity_log2 = 18;
  cfg->max_token_len = 255;
  cfg->inversion = TFIDF_INVERSION_AUTO;
  return TFIDF_OK;
}

extern "C" int tfidf_create(const tfidf_config *cfg, tfidf_index **out) {
  if (!cfg || !out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  if (cfg->max_token_len != 255) return fail(TFIDF_E_INVALID_ARG, "only max_token_len = 255 is supported");
  uint32_t lg = cfg->vocab_capacity_log2 ? cfg->vocab_capacity_log2 : 18;
  if (lg < 10 || lg > 26) return fail(TFIDF_E_INVALID_ARG, "vocab_capacity_log2 must be in [10, 26]");
  if (lg > kMaxBlockCapLog2 && cfg->inversion == TFIDF_INVERSION_BLOCK)
    return fail(TFIDF_E_INVALID_ARG, "block-major inversion supports vocab_capacity_log2 <= %u", kMaxBlockCapLog2);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(TFIDF_E_NO_DEVICE, "no HIP device");
  if (cfg->device < 0 || cfg->device >= ndev) return fail(TFIDF_E_NO_DEVICE, "device %d out of range", cfg->device);
  DeviceGuard g(cfg->device);
  tfidf_index *ix = new tfidf_index();
  ix->cfg = *cfg;
  ix->cfg.vocab_capacity_log2 = lg;
  ix->cap_log2 = lg;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, cfg->device) == hipSuccess) ix->num_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&ix->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete ix;
    return fail(TFIDF_E_HIP, "hipStreamCreate failed");
  }
  ix->stream = ix->own_stream;
  if (const char *cm = knob("TFIDF_COALESCE_MAX")) ix->cq_max = std::max(1, atoi(cm));   // tests: small batches
  if (hipStreamCreateWithFlags(&ix->copy_stream, hipStreamNonBlocking) != hipSuccess) {
    hipStreamDestroy(ix->own_stream);
    delete ix;
    return fail(TFIDF_E_HIP, "hipStreamCreate failed");
  }
  for (int i = 0; i < EV_N; i++) hipEventCreate(&ix->ev[i]);
  for (int i = 0; i < 2; i++) hipEventCreateWithFlags(&ix->stage_ev[i], hipEventDisableTiming);
  for (int i = 0; i < 3; i++) hipEventCreateWithFlags(&ix->mir_ev[i], hipEventDisableTiming);
  ix->text = std::make_shared<DevMem>(cfg->device);
  ix->offsets = std::make_shared<DevMem>(cfg->device);
  hipError_t e = ix->offsets->reserve(64);
  if (e != hipSuccess) { delete ix; return fail(TFIDF_E_OOM, "hipMalloc offsets"); }
  uint64_t zero = 0;
  hipMemcpy(ix->offsets->p, &zero, 8, hipMemcpyHostToDevice);
  *out = ix;
  return TFIDF_OK;
}

extern "C" int tfidf_destroy(tfidf_index *ix) {
  if (!ix) return TFIDF_OK;
  DeviceGuard g(ix->cfg.device);
  hipStreamSynchronize(ix->stream);
  hipStreamSynchronize(ix->copy_stream);
  ix->cur.reset();
  ix->spare.reset();
  ix->ctx_free.clear();
  ix->text.reset();
  ix->offsets.reset();
  DevBuf *bufs[] = {&ix->d_live_map, &ix->long_list, &ix->uni_list, &ix->counters, &ix->retry_list, &ix->bad_list,
                    &ix->post_tmp, &ix->lt_keys, &ix->lt_cnt, &ix->lt_g, &ix->lt_pos, &ix->verify_defer, &ix->pairs,
                    &ix->pair_ub, &ix->chunk_list, &ix->chunk_docs, &ix->chunk_fail, &ix->uchunk, &ix->canon_of_slot,
                    &ix->tvals, &ix->term_tmp, &ix->term_esc, &ix->sent_slot, &ix->vcounts, &ix->vnu, &ix->vt_table,
                    &ix->vt_sum, &ix->vt_rslot, &ix->gdf_dev};
  for (DevBuf *b : bufs) b->release();
  for (int i = 0; i < EV_N; i++) hipEventDestroy(ix->ev[i]);
  for (int i = 0; i < 2; i++) {
    if (ix->stage[i]) hipHostFree(ix->stage[i]);
    hipEventDestroy(ix->stage_ev[i]);
  }
  for (int i = 0; i < 3; i++) hipEventDestroy(ix->mir_ev[i]);
  hipStreamSynchronize(ix->own_stream);
  hipStreamDestroy(ix->copy_stream);
  hipStreamDestroy(ix->own_stream);
  delete ix;
  return TFIDF_OK;
}

// grow a device buffer shared with published snapshots: a new buffer with the
// first `keep` bytes copied (the snapshots keep the old one alive)
static int grow_shared(tfidf_index *ix, std::shared_ptr<DevMem> *buf, uint64_t need, uint64_t keep, bool zero) {
  if (need <= (*buf)->bytes) return TFIDF_OK;
  uint64_t cap = (*buf)->bytes ? (*buf)->bytes : (1ull << 20);
  while (cap < need) cap = cap + cap / 2 + (1ull << 20);
  auto nb = std::make_shared<DevMem>(ix->cfg.device);
  HIP_TRY(nb->reserve(cap));
  if (zero) HIP_TRY(hipMemsetAsync(nb->p, 0, cap, ix->stream));
  if ((*buf)->p && keep) HIP_TRY(hipMemcpyAsync(nb->p, (*buf)->p, keep, hipMemcpyDeviceToDevice, ix->stream));
  HIP_TRY(hipStreamSynchronize(ix->stream));
  *buf = std::move(nb);
  return TFIDF_OK;
}

// grow the device corpus to hold `extra` more bytes (plus read slack)
static int grow_text(tfidf_index *ix, uint64_t extra) {
  return grow_shared(ix, &ix->text, ix->text_bytes + extra + 128, ix->text_bytes, true);
}

static int grow_offsets(tfidf_index *ix, uint64_t extra_docs) {
  return grow_shared(ix, &ix->offsets, (ix->n_staged + extra_docs + 1) * 8, (ix->n_staged + 1) * 8, false);
}

static void register_key(tfidf_index *ix, const uint8_t *k, uint64_t n, bool synth) {
  const uint64_t idx = ix->n_staged;
  KeyChunk &c = ix->keys.tail(idx);
  if (!synth) {
    std::string key((const char *)k, n);
    auto it = ix->key_to_staged.find(key);
    if (it != ix->key_to_staged.end()) {       // updateDocument: delete-by-term, then add
      if (ix->staged_live[it->second]) { ix->staged_live[it->second] = 0; ix->n_dead++; }
      it->second = idx;
    } else {
      ix->key_to_staged.emplace(std::move(key), idx);
    }
    c.arena.append((const char *)k, n);
  }
  c.off.push_back(c.arena.size());
  c.synth.push_back(synth ? 1 : 0);
  ix->staged_live.push_back(1);
}

// Corpus loader (replaces Worker.init's per-file
// Files.readString + IndexWriter feed, J/worker/Worker.java:77-86,198): host
// bytes are copied into one of two pinned staging buffers by a few host
// threads while the other buffer's DMA to HBM is in flight, so the PCIe link
// streams at DMA speed instead of through the runtime's pageable bounce path.
constexpr size_t kStageBytes = 32u << 20;

static void par_memcpy(uint8_t *dst, const uint8_t *src, size_t n) {
  const size_t kMinPer = 4u << 20;
  unsigned t = std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency()));
  t = (unsigned)std::min<size_t>(t, std::max<size_t>(1, n / kMinPer));
  if (t <= 1) { memcpy(dst, src, n); return; }
  std::vector<std::thread> th;
  const size_t per = (n + t - 1) / t;
  for (unsigned i = 1; i < t; i++) {
    const size_t a = i * per, z = std::min(n, a + per);
    if (a < z) th.emplace_back([=] { memcpy(dst + a, src + a, z - a); });
  }
  memcpy(dst, src, std::min(n, per));
  for (auto &x : th) x.join();
}

static hipError_t h2d_staged(tfidf_index *ix, uint8_t *dst, const uint8_t *src, uint64_t n) {
  if (n < (1u << 20)) return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, ix->stream);
  for (int i = 0; i < 2; i++)
    if (!ix->stage[i]) {
      hipError_t e = hipHostMalloc(&ix->stage[i], kStageBytes, hipHostMallocDefault);
      if (e != hipSuccess) { ix->stage[i] = nullptr; return e; }
    }
  uint64_t off = 0;
  for (int c = 0; off < n; c++) {
    const int b = c & 1;
    const size_t sz = (size_t)std::min<uint64_t>(kStageBytes, n - off);
    hipError_t e = hipEventSynchronize(ix->stage_ev[b]);     // this buffer's previous DMA is done
    if (e != hipSuccess) return e;
    par_memcpy(static_cast<uint8_t *>(ix->stage[b]), src + off, sz);
    e = hipMemcpyAsync(dst + off, ix->stage[b], sz, hipMemcpyHostToDevice, ix->stream);
    if (e != hipSuccess) return e;
    e = hipEventRecord(ix->stage_ev[b], ix->stream);
    if (e != hipSuccess) return e;
    off += sz;
  }
  return hipSuccess;
}

extern "C" int tfidf_clear(tfidf_index *ix) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard g(ix->cfg.device);
  HIP_TRY(hipStreamSynchronize(ix->stream));
  // The staged corpus restarts at offset 0: buffers a published snapshot (an
  // open reader, an in-flight search) still reads are replaced, not rewritten.
  if (ix->text.use_count() > 1) ix->text = std::make_shared<DevMem>(ix->cfg.device);
  if (ix->offsets.use_count() > 1) {
    auto no = std::make_shared<DevMem>(ix->cfg.device);
    HIP_TRY(no->reserve(64));
    HIP_TRY(hipMemsetAsync(no->p, 0, 8, ix->stream));
    HIP_TRY(hipStreamSynchronize(ix->stream));
    ix->offsets = std::move(no);
  }
  ix->text_bytes = 0;
  ix->n_staged = 0;
  ix->h_offsets.assign(1, 0);
  ix->keys = KeyTable();
  ix->staged_live.clear();
  ix->key_to_staged.clear();
  ix->n_dead = 0;
  std::shared_ptr<Snapshot> old;
  {
    std::lock_guard<std::mutex> sl(ix->snap_mu);    // searches from now on: not committed
    old = std::move(ix->cur);
  }
  if (!ix->spare) ix->spare = std::move(old);       // buffers for the next commit
  return TFIDF_OK;
}

// ---------------------------------------------------------------------------
// Persistence (the reference keeps a Lucene index in
// FSDirectory(lucene.index.path) and reopens it at start-up,
// J/worker/Worker.java:67-73).  What is stored is the staged corpus (text,
// offsets, document keys, liveness after replace-by-key) — the index
// structures are rebuilt by tfidf_commit on load: on MI355X the rebuild runs
// at tens of GB/s of corpus, faster than reading the derived structures
// (≈ 2x the corpus size) back from storage.
static const char kFileMagic[8] = {'T', 'F', 'I', 'D', 'F', 'I', 'X', '1'};

struct FileHeader {
  char magic[8];
  uint32_t version, reserved;
  float k1, b;
  int32_t stats_mode, inversion;
  uint32_t vocab_capacity_log2, pad;
  uint64_t n_staged, text_bytes, key_bytes, n_dead, meta_hash;
};

static uint64_t fnv1a(uint64_t h, const void *p, size_t n) {
  const uint8_t *c = static_cast<const uint8_t *>(p);
  for (size_t i = 0; i < n; i++) { h ^= c[i]; h *= 0x100000001B3ull; }
  return h;
}

static uint64_t meta_hash(const tfidf_index *ix, const std::string &arena, const std::vector<uint64_t> &koff,
                          const std::vector<uint8_t> &synth) {
  uint64_t h = 0xCBF29CE484222325ull;
  h = fnv1a(h, ix->h_offsets.data(), ix->h_offsets.size() * 8);
  h = fnv1a(h, koff.data(), koff.size() * 8);
  h = fnv1a(h, arena.data(), arena.size());
  h = fnv1a(h, synth.data(), synth.size());
  h = fnv1a(h, ix->staged_live.data(), ix->staged_live.size());
  return h;
}

extern "C" int tfidf_save(tfidf_index *ix, const char *path) {
  if (!ix || !path) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard g(ix->cfg.device);
  HIP_TRY(hipStreamSynchronize(ix->stream));
  std::string key_arena;
  std::vector<uint64_t> key_off;
  std::vector<uint8_t> key_synth;
  ix->keys.flatten(&key_arena, &key_off, &key_synth);
  FileHeader h{};
  memcpy(h.magic, kFileMagic, 8);
  h.version = 1;
  h.k1 = ix->cfg.k1;
  h.b = ix->cfg.b;
  h.stats_mode = ix->cfg.stats_mode;
  h.inversion = ix->cfg.inversion;
  h.vocab_capacity_log2 = ix->cap_log2;
  h.n_staged = ix->n_staged;
  h.text_bytes = ix->text_bytes;
  h.key_bytes = key_arena.size();
  h.n_dead = ix->n_dead;
  h.meta_hash = meta_hash(ix, key_arena, key_off, key_synth);
  const std::string tmp = std::string(path) + ".tmp";
  FILE *f = fopen(tmp.c_str(), "wb");
  if (!f) return fail(TFIDF_E_INVALID_ARG, "cannot open %s for writing", tmp.c_str());
  bool ok = fwrite(&h, sizeof h, 1, f) == 1;
  ok = ok && fwrite(ix->h_offsets.data(), 8, ix->h_offsets.size(), f) == ix->h_offsets.size();
  ok = ok && fwrite(key_off.data(), 8, key_off.size(), f) == key_off.size();
  ok = ok && (key_arena.empty() || fwrite(key_arena.data(), 1, key_arena.size(), f) == key_arena.size());
  ok = ok && (ix->n_staged == 0 || fwrite(key_synth.data(), 1, ix->n_staged, f) == ix->n_staged);
  ok = ok && (ix->n_staged == 0 || fwrite(ix->staged_live.data(), 1, ix->n_staged, f) == ix->n_staged);
  // corpus text: device -> pinned staging buffer -> file, chunk by chunk
  if (ok && ix->text_bytes) {
    if (!ix->stage[0]) {
      if (hipHostMalloc(&ix->stage[0], kStageBytes, hipHostMallocDefault) != hipSuccess) ix->stage[0] = nullptr;
    }
    if (!ix->stage[0]) { fclose(f); remove(tmp.c_str()); return fail(TFIDF_E_OOM, "pinned staging buffer"); }
    for (uint64_t off = 0; ok && off < ix->text_bytes; off += kStageBytes) {
      const size_t n = (size_t)std::min<uint64_t>(kStageBytes, ix->text_bytes - off);
      if (hipMemcpy(ix->stage[0], ix->text->as<uint8_t>() + off, n, hipMemcpyDeviceToHost) != hipSuccess) {
        fclose(f);
        remove(tmp.c_str());
        return fail(TFIDF_E_HIP, "copy of the corpus from the device failed");
      }
      ok = fwrite(ix->stage[0], 1, n, f) == n;
    }
  }
  ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), path) != 0) {
    remove(tmp.c_str());
    return fail(TFIDF_E_INVALID_ARG, "write of %s failed", path);
  }
  return TFIDF_OK;
}

extern "C" int tfidf_add_docs(tfidf_index *ix, const uint8_t *utf8, const uint64_t *offsets, uint64_t n_docs,
                              const uint8_t *keys, const uint64_t *key_offsets);

extern "C" int tfidf_load(tfidf_index *ix, const char *path) {
  if (!ix || !path) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  {
    std::lock_guard<std::mutex> lk(ix->mu);
    if (ix->n_staged) return fail(TFIDF_E_STATE, "tfidf_load needs an empty index (tfidf_create / tfidf_clear)");
  }
  FILE *f = fopen(path, "rb");
  if (!f) return fail(TFIDF_E_INVALID_ARG, "cannot open %s", path);
  FileHeader h{};
  if (fread(&h, sizeof h, 1, f) != 1 || memcmp(h.magic, kFileMagic, 8) != 0 || h.version != 1) {
    fclose(f);
    return fail(TFIDF_E_INVALID_ARG, "%s is not a tfidf index file (version 1)", path);
  }
  if (h.vocab_capacity_log2 != ix->cap_log2) {
    fclose(f);
    return fail(TFIDF_E_INVALID_ARG, "index file has vocab_capacity_log2 %u, this index %u", h.vocab_capacity_log2,
                ix->cap_log2);
  }
  const uint64_t n = h.n_staged;
  std::vector<uint64_t> offs(n + 1), koff(n + 1);
  std::string arena(h.key_bytes, '\0');
  std::vector<uint8_t> synth(n), live(n);
  bool ok = fread(offs.data(), 8, n + 1, f) == n + 1 && fread(koff.data(), 8, n + 1, f) == n + 1;
  ok = ok && (h.key_bytes == 0 || fread(&arena[0], 1, h.key_bytes, f) == h.key_bytes);
  ok = ok && (n == 0 || (fread(synth.data(), 1, n, f) == n && fread(live.data(), 1, n, f) == n));
  ok = ok && offs[0] == 0 && offs[n] == h.text_bytes && koff[0] == 0 && koff[n] == h.key_bytes;
  for (uint64_t i = 0; ok && i < n; i++) ok = offs[i + 1] >= offs[i] && koff[i + 1] >= koff[i];
  std::vector<uint8_t> text;
  if (ok) {
    text.resize(h.text_bytes);
    ok = h.text_bytes == 0 || fread(text.data(), 1, h.text_bytes, f) == h.text_bytes;
  }
  fclose(f);
  if (!ok) return fail(TFIDF_E_INVALID_ARG, "%s is truncated or corrupt", path);
  // stage every stored document (as if keyless), then restore keys and
  // liveness exactly as saved
  int rc = tfidf_add_docs(ix, n ? text.data() : nullptr, offs.data(), n, nullptr, nullptr);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ix->mu);
  {
    auto one = std::make_shared<KeyChunk>();
    one->arena = arena;
    one->off.assign(koff.begin(), koff.end());
    one->synth = synth;
    ix->keys.ch.assign(1, one);
  }
  ix->staged_live = live;
  ix->key_to_staged.clear();
  ix->n_dead = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (!live[i]) { ix->n_dead++; continue; }
    if (!synth[i]) ix->key_to_staged[std::string(arena, koff[i], koff[i + 1] - koff[i])] = i;
  }
  if (ix->n_dead != h.n_dead || meta_hash(ix, arena, koff, synth) != h.meta_hash) {
    return fail(TFIDF_E_INVALID_ARG, "%s: metadata checksum mismatch", path);
  }
  return TFIDF_OK;
}

extern "C" int tfidf_add_docs(tfidf_index *ix, const uint8_t *utf8, const uint64_t *offsets, uint64_t n_docs,
                              const uint8_t *keys, const uint64_t *key_offsets) {
  if (!ix || (!utf8 && n_docs) || !offsets) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  if (keys && !key_offsets) return fail(TFIDF_E_INVALID_ARG, "keys without key_offsets");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard g(ix->cfg.device);
  for (uint64_t i = 0; i < n_docs; i++)
    if (offsets[i + 1] < offsets[i]) return fail(TFIDF_E_INVALID_ARG, "offsets must be non-decreasing");
  const uint64_t nbytes = offsets[n_docs] - offsets[0];
  if (ix->n_staged + n_docs >= 0xFFFFFFF0ull) return fail(TFIDF_E_CAPACITY, "more than 2^32 documents per shard");
  int rc = grow_text(ix, nbytes);
  if (rc) return rc;
  rc = grow_offsets(ix, n_docs);
  if (rc) return rc;
  if (nbytes) HIP_TRY(h2d_staged(ix, ix->text->as<uint8_t>() + ix->text_bytes, utf8 + offsets[0], nbytes));
  std::vector<uint64_t> no(n_docs);
  for (uint64_t i = 0; i < n_docs; i++) no[i] = ix->text_bytes + (offsets[i + 1] - offsets[0]);
  if (n_docs)
    HIP_TRY(hipMemcpyAsync(ix->offsets->as<uint64_t>() + ix->n_staged + 1, no.data(), n_docs * 8,
                           hipMemcpyHostToDevice, ix->stream));
  HIP_TRY(hipStreamSynchronize(ix->stream));
  for (uint64_t i = 0; i < n_docs; i++) {
    if (keys) register_key(ix, keys + key_offsets[i], key_offsets[i + 1] - key_offsets[i], false);
    else register_key(ix, nullptr, 0, true);
    ix->h_offsets.push_back(no[i]);
    ix->n_staged++;
  }
  ix->text_bytes += nbytes;                 // searches keep the last commit's snapshot
  return TFIDF_OK;
}

extern "C" int tfidf_add_docs_device(tfidf_index *ix, const void *d_utf8, const void *d_offsets, uint64_t n_docs,
                                     uint64_t total_bytes) {
  if (!ix || !d_offsets) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard g(ix->cfg.device);
  if (ix->n_staged + n_docs >= 0xFFFFFFF0ull) return fail(TFIDF_E_CAPACITY, "more than 2^32 documents per shard");
  std::vector<uint64_t> ho(n_docs + 1);
  HIP_TRY(hipMemcpy(ho.data(), d_offsets, (n_docs + 1) * 8, hipMemcpyDeviceToHost));
  if (ho[n_docs] - ho[0] != total_bytes) return fail(TFIDF_E_INVALID_ARG, "total_bytes != offsets[n] - offsets[0]");
  int rc = grow_text(ix, total_bytes);
  if (rc) return rc;
  rc = grow_offsets(ix, n_docs);
  if (rc) return rc;
  if (total_bytes)
    HIP_TRY(hipMemcpyAsync(ix->text->as<uint8_t>() + ix->text_bytes, (const uint8_t *)d_utf8 + ho[0], total_bytes,
                           hipMemcpyDeviceToDevice, ix->stream));
  uint64_t *dst = ix->offsets->as<uint64_t>() + ix->n_staged + 1;
  HIP_TRY(hipMemcpyAsync(dst, (const uint64_t *)d_offsets + 1, n_docs * 8, hipMemcpyDeviceToDevice, ix->stream));
  HIP_TRY(add_u64(dst, n_docs, ix->text_bytes - ho[0], ix->stream));
  HIP_TRY(hipStreamSynchronize(ix->stream));
  for (uint64_t i = 0; i < n_docs; i++) {
    register_key(ix, nullptr, 0, true);
    ix->h_offsets.push_back(ix->text_bytes + (ho[i + 1] - ho[0]));
    ix->n_staged++;
  }
  ix->text_bytes += total_bytes;
  return TFIDF_OK;
}

// BM25 norm cache for the statistics in force (BM25Similarity.scorer, float ops)
static void norm_cache(float k1, float b, float avgdl, float *cache) {
  for (int i = 0; i < 256; i++) {
    volatile float len = (float)byte4_to_int((uint32_t)i);
    volatile float t1 = 1.0f - b;
    volatile float t2 = b * len;
    volatile float t3 = t2 / avgdl;
    volatile float t4 = t1 + t3;
    volatile float t5 = k1 * t4;
    cache[i] = 1.0f / t5;
  }
}

static float bm25_idf(uint64_t df, uint64_t doc_count) {
  const double x = ((double)((int64_t)doc_count - (int64_t)df) + 0.5) / ((double)df + 0.5);
  return (float)log(1.0 + x);
}

// BM25 norm cache of a statistics view (not yet visible to searches, or
// owned by the writer), uploaded on stream s.  sync = false: the caller
// guarantees no earlier upload out of v.h_cache is pending and orders the
// view's first use after this one (StatsView::gdf_ev).
static int upload_cache(const tfidf_config &cfg, StatsView &v, hipStream_t s, bool sync = true) {
  HIP_TRY(v.h_cache.resize(256));
  // the previous upload from the staging array must be done before it is rewritten
  if (sync) HIP_TRY(hipStreamSynchronize(s));
  float *c = v.h_cache.data();
  if (v.doc_count == 0) {
    for (int i = 0; i < 256; i++) c[i] = 0.0f;
  } else {
    const float avgdl = (float)((double)v.sum_ttf / (double)v.doc_count);
    norm_cache(cfg.k1, cfg.b, avgdl, c);
  }
  HIP_TRY(v.cache.reserve(256 * 4));
  HIP_TRY(hipMemcpyAsync(v.cache.p, c, 256 * 4, hipMemcpyHostToDevice, s));
  if (sync) HIP_TRY(hipStreamSynchronize(s));
  return TFIDF_OK;
}

static float ev_ms(tfidf_index *ix, int a, int b) {
  float ms = 0;
  hipEventElapsedTime(&ms, ix->ev[a], ix->ev[b]);
  return ms;
}

static float qev_ms(const SearchCtx &c, int a, int b) {
  float ms = 0;
  if (!c.q_timing) return -1.0f;                   // query timing off: not measured
  hipEventElapsedTime(&ms, c.ev[a], c.ev[b]);
  return ms;
}

static void set_last_ms(tfidf_index *ix, float scoring, float total) {
  std::lock_guard<std::mutex> lk(ix->ms_mu);
  ix->last_ms_scoring = scoring;
  ix->last_ms_total = total;
}

// One index build with ix->hash_seed; kRcCollision when two different terms
// met under one hashed key (tfidf_commit then rebuilds with another seed).
constexpr int kRcCollision = -1000;
constexpr int kRcNoPublish = -1001;             // TFIDF_DEBUG_STOP (profiling): the rows are incomplete
constexpr uint32_t kVerifyCap = 1u << 20;      // deferred hashed-key checks per build
static int commit_once(tfidf_index *ix, Snapshot &S) {
  hipStream_t s = ix->stream;
  // live documents
  S.n_docs = ix->n_staged - ix->n_dead;
  S.live_map.clear();
  if (ix->n_dead) {
    S.live_map.reserve(S.n_docs);
    for (uint64_t i = 0; i < ix->n_staged; i++)
      if (ix->staged_live[i]) S.live_map.push_back((uint32_t)i);
    HIP_TRY(ix->d_live_map.reserve(S.n_docs * 4 + 4));
    HIP_TRY(hipMemcpyAsync(ix->d_live_map.p, S.live_map.data(), S.n_docs * 4, hipMemcpyHostToDevice, s));
  }
  const uint64_t N = S.n_docs;
  S.C = 1u << ix->cap_log2;
  const uint32_t C = S.C;
  S.n_blocks = (uint32_t)((N + kBlockDocs - 1) / kBlockDocs);
  const uint64_t row_cap = (ix->text_bytes + ix->n_staged) / 2 + 2;
  // Inversion layout: block-major needs a dense (blocks + 1) x C count table;
  // when that outgrows the CSR itself (huge vocabularies, SURVEY §8 cfg 5) the
  // postings are built term-major by a sort instead (kernels_term.hip).
  {
    const uint64_t blk_bytes = (uint64_t)(S.n_blocks + 1) * C * 4;
    if (ix->cfg.inversion == TFIDF_INVERSION_TERM) S.term_major = true;
    else if (ix->cfg.inversion == TFIDF_INVERSION_BLOCK) S.term_major = false;
    else {
      // Few (block, range) tiles of very long documents (a few hundred books,
      // SURVEY cfg 1): the block-major passes run one workgroup per tile and
      // starve; the sort-based term-major build is parallel in the postings.
      const uint64_t tiles = (uint64_t)S.n_blocks * (C < kRangeSlots ? 1u : C / kRangeSlots);
      const bool starved = tiles < ix->num_cus && ix->n_staged && ix->text_bytes / ix->n_staged >= (64u << 10);
      S.term_major = ix->cap_log2 > kMaxBlockCapLog2 || (blk_bytes > (1ull << 31) && blk_bytes > row_cap * 4) ||
                       starved;
    }
  }
  // CSR rows are grouped by dictionary range for the block-major passes only
  const uint32_t RS = S.term_major ? C : (C < kRangeSlots ? C : kRangeSlots);
  S.range_shift = 0;
  while ((1u << S.range_shift) < RS) S.range_shift++;
  S.R = C >> S.range_shift;

  HIP_TRY(S.dict.reserve((size_t)3 * C * 8));          // lo, hi, reference occurrence (dict_device.h)
  HIP_TRY(ix->verify_defer.reserve((size_t)kVerifyCap * 16));
  HIP_TRY(S.csr.reserve(row_cap * 4));
  // escapes: each needs tf >= the field's escape value, and a row holds at
  // most row_cap tokens in all, so this bounds their number
  const uint64_t esc_cap = row_cap / csr_esc_value(S.range_shift) + 64;
  HIP_TRY(S.csr_esc.reserve(esc_cap * 8));
  HIP_TRY(S.doc_len.reserve(N * 4 + 4));
  HIP_TRY(S.doc_nuniq.reserve(N * 4 + 4));
  HIP_TRY(S.doc_norm.reserve(N + 16));
  HIP_TRY(S.rsplit.reserve(N * S.R * 4 + 4));
  HIP_TRY(ix->long_list.reserve(N * 4 + 4));
  HIP_TRY(ix->uni_list.reserve(N * 4 + 4));
  HIP_TRY(ix->counters.reserve(128));
  HIP_TRY(ix->bad_list.reserve(N * 4 + 4));
  // Short-document corpora: the wave path indexes packs of consecutive
  // documents per window (about kPackBytes of text per pack; SURVEY cfg 5
  // shape: 6 documents of ~330 B).  TFIDF_PACK_DOCS overrides (tests).
  uint32_t pack = 1;
  {
    const uint64_t avg = ix->n_staged ? ix->text_bytes / ix->n_staged : 0;
    if (avg) pack = (uint32_t)std::min<uint64_t>(kPackMaxDocs, std::max<uint64_t>(1, kPackBytes / avg));
    if (const char *e = knob("TFIDF_PACK_DOCS")) pack = (uint32_t)std::max(1, std::min(atoi(e), (int)kPackMaxDocs));
    pack = std::min(pack, std::max(1u, kWaveGroups / S.R));   // (document, range) groups per unit
  }
  if (pack > 1) HIP_TRY(ix->retry_list.reserve(N * 4 + 4));
  if (S.term_major) {
    HIP_TRY(S.row_off.reserve(N * 4 + 4));
    HIP_TRY(S.toff.reserve(((size_t)C + 1) * 8));
    HIP_TRY(S.tdf.reserve((size_t)C * 4));
  } else {
    // (the count table blk is sized by the columns, known after the tokenizers)
    HIP_TRY(S.bbase.reserve((size_t)(S.n_blocks + 2) * 8));
    HIP_TRY(S.crank.reserve(((size_t)C / 32 + 1) * 8));
    HIP_TRY(S.sdf.reserve((size_t)C * 4));
  }

  // counters: [0..2] stats u64, [3] err flags u32 + [3].hi first doc, [4] long_count, [5] retry_count,
  // [6] uni_count, [7] occupied dictionary slots, [8] bad_count, [9] CSR escape count, [10] posting
  // escapes, [11] deferred hashed-key checks, [12] term-major tf escapes, [13] flagged documents
  // the wave rules took (k_tokenize_wave<UNI>)
  uint64_t *ctr = ix->counters.as<uint64_t>();
  HIP_TRY(hipMemsetAsync(ix->counters.p, 0, 128, s));
  HIP_TRY(hipMemsetAsync(S.dict.p, 0, (size_t)3 * C * 8, s));
  // per-document Unicode flags.  UNI-first (the last commit's documents were
  // mostly non-ASCII, one document per wave): every document starts flagged
  // and k_tokenize_wave<UNI> takes ASCII ones as well, so the ASCII pass —
  // which would only read each such document to flag it — does not run
  // (cfg-2 prose: 0.8 ms)
  const char *nouw = knob("TFIDF_NO_UNIWAVE");
  const bool uni_on = !(nouw && *nouw && *nouw != '0');
  const bool uni_first = ix->uni_first && uni_on && pack == 1 && !knob("TFIDF_NO_UNIFIRST");
  if (uni_first) HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)ix->uni_list.p, 1u, N, s));
  else HIP_TRY(hipMemsetAsync(ix->uni_list.p, 0, (size_t)N * 4, s));

  BuildParams bp{};
  bp.text = ix->text->as<uint8_t>();
  bp.offsets = ix->offsets->as<uint64_t>();
  bp.live_map = ix->n_dead ? ix->d_live_map.as<uint32_t>() : nullptr;
  bp.n_docs = N;
  bp.dict = S.dict.as<uint64_t>();
  bp.cap_mask = C - 1;
  bp.range_shift = S.range_shift;
  bp.n_ranges = S.R;
  bp.hash_seed = ix->hash_seed;
  bp.verify_defer = ix->verify_defer.as<uint64_t>();
  bp.verify_count = reinterpret_cast<uint32_t *>(ctr + 11);
  bp.verify_cap = kVerifyCap;
  bp.csr = S.csr.as<uint32_t>();
  bp.csr_esc = S.csr_esc.as<uint64_t>();
  bp.esc_count = reinterpret_cast<uint32_t *>(ctr + 9);
  bp.esc_cap = esc_cap;
  bp.doc_len = S.doc_len.as<uint32_t>();
  bp.doc_nuniq = S.doc_nuniq.as<uint32_t>();
  bp.doc_norm = S.doc_norm.as<uint8_t>();
  bp.rsplit = S.rsplit.as<uint32_t>();
  bp.long_list = ix->long_list.as<uint32_t>();
  bp.long_count = reinterpret_cast<uint32_t *>(ctr + 4);
  bp.uni_list = ix->uni_list.as<uint32_t>();
  bp.uni_count = reinterpret_cast<uint32_t *>(ctr + 6);
  bp.uni_wave_count = reinterpret_cast<uint32_t *>(ctr + 13);
  bp.bad_list = ix->bad_list.as<uint32_t>();
  bp.bad_count = reinterpret_cast<uint32_t *>(ctr + 8);
  bp.stats = reinterpret_cast<unsigned long long *>(ctr);
  bp.err = reinterpret_cast<uint32_t *>(ctr + 3);
  if (const char *ds = knob("TFIDF_DEBUG_STOP")) bp.debug_stop = (uint32_t)atoi(ds);   // profiling only
  if (const char *uf = knob("TFIDF_UW_FULL")) bp.debug_uw_full = (uint32_t)atoi(uf);   // A/B only
  bp.pack = pack;
  bp.retry_list = pack > 1 ? ix->retry_list.as<uint32_t>() : nullptr;
  bp.retry_count = reinterpret_cast<uint32_t *>(ctr + 5);
  S.pack_docs = pack;
  S.pack_retried = 0;

  HIP_TRY(hipEventRecord(ix->ev[EV_START], s));
  if (N) {
    const uint64_t units = (N + pack - 1) / pack;
    uint64_t wpc = kWaveWGsPerCU;
    if (const char *e = knob("TFIDF_WAVE_WGS_PER_CU")) wpc = (uint64_t)std::max(1, atoi(e));   // profiling only
    const uint64_t grid = std::min<uint64_t>(units, (uint64_t)ix->num_cus * wpc);
    if (!uni_first) HIP_TRY(launch_tokenize_wave(bp, (int)grid, s));
    if (pack > 1 && !bp.debug_stop) {       // documents the packs could not take: one per wave
      uint32_t n_retry = 0;
      HIP_TRY(hipMemcpyAsync(&n_retry, ctr + 5, 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      S.pack_retried = n_retry;
      if (n_retry) {
        BuildParams rp = bp;
        rp.pack = 1;
        rp.doc_list = bp.retry_list;
        rp.doc_list_count = bp.retry_count;
        const uint64_t rgrid = std::min<uint64_t>(n_retry, (uint64_t)ix->num_cus * kWaveWGsPerCU);
        HIP_TRY(launch_tokenize_wave(rp, (int)rgrid, s));
      }
    }
    // documents with non-ASCII text (flags read on the device; both exit at once
    // when none): the wave rules with non-ASCII letters where the document's
    // characters allow (k_tokenize_wave<UNI>), then the Unicode wave path for
    // the rest.  TFIDF_NO_UNIWAVE: the Unicode wave path for all (A/B).
    if (bp.debug_stop < 10 && uni_on)
      HIP_TRY(launch_tokenize_wave_uni(bp, (int)std::min<uint64_t>((N + 63) / 64, (uint64_t)ix->num_cus * kWaveWGsPerCU), s));
    if (!bp.debug_stop || bp.debug_stop >= 10)          // (stops 10..13: the Unicode wave path's phases)
      HIP_TRY(launch_tokenize_uwave(bp, (int)std::min<uint64_t>(N, (uint64_t)ix->num_cus * kUwaveWGsPerCU), s));
  }
  HIP_TRY(hipEventRecord(ix->ev[EV_TOK], s));
  if (bp.debug_stop) {                      // profiling only: rows are incomplete, stop here
    HIP_TRY(hipStreamSynchronize(s));
    ix->timing = tfidf_commit_timing{};
    ix->timing.ms_tokenize = ev_ms(ix, EV_START, EV_TOK);
    ix->timing.ms_total = ix->timing.ms_tokenize;
    ix->timing.text_bytes = ix->text_bytes;
    ix->timing.num_docs = N;
    return kRcNoPublish;
  }
  // block-major: columns of the dictionary as it stands (final unless the
  // long path runs below, which recomputes them); their count lands in ctr[7]
  auto col_rank = [&]() -> int {
    if (!S.term_major)
      HIP_TRY(launch_col_rank(S.dict.as<uint64_t>(), C, S.crank.as<uint2>(),
                              reinterpret_cast<unsigned long long *>(ctr + 7), s));
    return TFIDF_OK;
  };
  if (int rc = col_rank()) return rc;
  // one read of the counters: stats (0-2), error flags (3), long (4) and
  // non-ASCII (6) document counts, columns (7), CSR escapes (9) (32-bit
  // counters in the low halves); read again only when the long path ran
  HIP_TRY(ix->hctr_h.resize(14));                      // pinned: a pageable read is staged by the runtime
  uint64_t *hctr = ix->hctr_h.data();
  HIP_TRY(hipMemcpyAsync(hctr, ctr, 14 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const uint32_t n_long = (uint32_t)hctr[4], n_uni = (uint32_t)hctr[6];
  S.long_chunked = 0;
  S.long_docs = n_long;
  S.unicode_docs = n_uni + (uint32_t)hctr[13];
  S.unicode_wave_docs = (uint32_t)hctr[13];
  ix->uni_first = pack == 1 && (uint64_t)S.unicode_docs * 2 > N;
  if (n_long) {
    HIP_TRY(hipEventRecord(ix->ev[EV_L0], s));
    // book-sized documents: chunk-parallel (k_tokenize_chunk + k_long_rows),
    // in groups whose unit pair lists fit kPairBudget; documents a chunk
    // could not take come back in long_list for k_tokenize_long
    // pinned host buffers: pageable copies are staged synchronously by the runtime
    PinnedVec<uint32_t> &ldocs = ix->ldocs_h;
    HIP_TRY(ldocs.resize(n_long));
    HIP_TRY(hipMemcpyAsync(ldocs.data(), ix->long_list.p, (size_t)n_long * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // pair buckets: at most 64, each a whole number of k_long_rows' LDS windows
    const uint32_t wlog = std::min<uint32_t>(ix->cap_log2, kLrWinBits);
    const uint32_t bsh = std::max<uint32_t>(wlog, ix->cap_log2 > 6 ? ix->cap_log2 - 6 : 0);
    const uint32_t nb = 1u << (ix->cap_log2 - bsh);
    uint64_t unit_max = std::max<uint64_t>(1, kPairBudget / ((uint64_t)kPairWords * 4));
    if (const char *e = knob("TFIDF_TEST_PAIR_UNITS")) unit_max = std::max(1, atoi(e));   // tests: many groups
    // per group: the first unit (document, core) of each document, prefix form
    std::vector<uint32_t> pre;
    std::vector<uint64_t> gpre, gdoc;               // each group's prefix array offset and first document
    uint64_t acc = 0, max_units = 0;
    for (uint64_t i = 0; i < n_long; i++) {
      const uint64_t st = S.live_map.empty() ? ldocs[i] : S.live_map[ldocs[i]];
      const uint64_t L = ix->h_offsets[st + 1] - ix->h_offsets[st];
      const uint64_t units = (L + kLongCoreBytes - 1) / kLongCoreBytes;
      if (i == 0 || acc + units > unit_max) {
        if (i) { pre.push_back((uint32_t)acc); max_units = std::max(max_units, acc); }
        gpre.push_back(pre.size());
        gdoc.push_back(i);
        acc = 0;
      }
      pre.push_back((uint32_t)acc);
      acc += units;
      if (acc >= 0xFFFFFFFFull) return fail(TFIDF_E_CAPACITY, "too many document chunks");
    }
    pre.push_back((uint32_t)acc);
    max_units = std::max(max_units, acc);
    gdoc.push_back(n_long);
    HIP_TRY(ix->pairs.reserve(max_units * kPairWords * 4));
    HIP_TRY(ix->pair_ub.reserve(max_units * (nb + 1) * 4));
    HIP_TRY(ix->chunk_list.reserve(pre.size() * 4 + 8));
    HIP_TRY(ix->chunk_docs.reserve((size_t)n_long * 4));
    HIP_TRY(ix->chunk_fail.reserve((size_t)n_long * 4));
    HIP_TRY(ix->uchunk.reserve(max_units * 4 + 16));     // [0] count, [4 ..] per unit: non-ASCII text
    HIP_TRY(ix->pre_h.resize(pre.size()));
    memcpy(ix->pre_h.data(), pre.data(), pre.size() * 4);
    HIP_TRY(hipMemcpyAsync(ix->chunk_list.p, ix->pre_h.data(), pre.size() * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ix->chunk_docs.p, ix->long_list.p, (size_t)n_long * 4, hipMemcpyDeviceToDevice, s));
    HIP_TRY(hipMemsetAsync(ix->chunk_fail.p, 0, (size_t)n_long * 4, s));
    HIP_TRY(hipMemsetAsync(bp.long_count, 0, 4, s));                   // the fallback list restarts
    for (size_t gi = 0; gi < gpre.size(); gi++) {
      const uint64_t g0 = gdoc[gi], n = gdoc[gi + 1] - g0;
      BuildParams cp = bp;
      cp.chunk_pre = ix->chunk_list.as<uint32_t>() + gpre[gi];
      cp.n_group_docs = (uint32_t)n;
      cp.n_chunks = pre[gpre[gi] + n];
      cp.chunk_docs = ix->chunk_docs.as<uint32_t>() + g0;
      cp.chunk_fail = ix->chunk_fail.as<uint32_t>() + g0;
      cp.pairs = ix->pairs.as<uint32_t>();
      cp.pair_ub = ix->pair_ub.as<uint32_t>();
      cp.pair_bshift = bsh;
      cp.pair_nb = nb;
      // units with non-ASCII text: the Unicode chunk kernel (TFIDF_NO_UCHUNK: their
      // documents go to k_tokenize_long whole, as before round 4; A/B only)
      const bool uch = !knob("TFIDF_NO_UCHUNK");
      cp.uchunk_count = uch ? ix->uchunk.as<uint32_t>() : nullptr;
      cp.uchunk_list = uch ? ix->uchunk.as<uint32_t>() + 4 : nullptr;
      if (uch) HIP_TRY(hipMemsetAsync(ix->uchunk.p, 0, (size_t)(cp.n_chunks + 4) * 4, s));
      const uint64_t grid = std::min<uint64_t>(cp.n_chunks, (uint64_t)ix->num_cus * kWaveWGsPerCU);
      HIP_TRY(launch_tokenize_chunks(cp, (int)grid, s));
      // flagged units by the wave rules where their text allows (TFIDF_NO_UNIWAVE: all
      // of them to the Unicode chunk kernel; A/B only), then the rest
      const char *nouw = knob("TFIDF_NO_UNIWAVE");
      if (uch && !(nouw && *nouw && *nouw != '0')) HIP_TRY(launch_tokenize_chunks_uni(cp, (int)grid, s));
      if (uch)      // the count is read on the device: exits at once when no unit was listed
        HIP_TRY(launch_tokenize_uchunk(cp, (int)std::min<uint64_t>(cp.n_chunks, (uint64_t)ix->num_cus * kUchunkWGsPerCU), s));
      HIP_TRY(launch_long_rows(cp, (uint32_t)n, s));
    }
    uint32_t n_fb = 0;
    HIP_TRY(hipMemcpyAsync(&n_fb, bp.long_count, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    S.long_chunked = n_long - n_fb;
    if (n_fb) {
      uint32_t lg = ix->cap_log2 + 1;
      // table size needed by the longest long document (2x its token bound)
      uint64_t maxlen = 0;
      for (uint64_t d = 0; d < ix->n_staged; d++) maxlen = std::max(maxlen, ix->h_offsets[d + 1] - ix->h_offsets[d]);
      uint32_t need = 10;
      while (need < 22 && (1ull << need) < maxlen + 2) need++;
      lg = std::min(lg, need);
      ix->lt_log2 = lg;
      // one workgroup per long document, up to 2 per CU, within a scratch budget
      // (24 B per table slot per workgroup: key lo/hi, count, dictionary slot)
      const uint64_t per_wg = 24ull << lg;
      const uint64_t by_budget = std::max<uint64_t>(ix->lt_wgs, kLongScratchBudget / per_wg);
      const uint32_t wgs = (uint32_t)std::min<uint64_t>({(uint64_t)n_fb, (uint64_t)ix->num_cus * 2, by_budget});
      HIP_TRY(ix->lt_keys.reserve((size_t)wgs * 2 * (1ull << lg) * 8));
      HIP_TRY(ix->lt_cnt.reserve((size_t)wgs * (1ull << lg) * 4));
      HIP_TRY(ix->lt_pos.reserve((size_t)wgs * (1ull << lg) * 8));
      HIP_TRY(ix->lt_g.reserve((size_t)wgs * (1ull << lg) * 4));
      bp.lt_keys = ix->lt_keys.as<uint64_t>();
      bp.lt_cnt = ix->lt_cnt.as<uint32_t>();
      bp.lt_pos = ix->lt_pos.as<uint64_t>();
      bp.lt_g = ix->lt_g.as<uint32_t>();
      bp.lt_slots_log2 = lg;
      HIP_TRY(launch_tokenize_long(bp, (int)wgs, s));
    }
    HIP_TRY(hipEventRecord(ix->ev[EV_LONG], s));
    if (int rc = col_rank()) return rc;
    HIP_TRY(hipMemcpyAsync(hctr, ctr, 10 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  const uint32_t err = (uint32_t)(hctr[3] & 0xFFFFFFFFu), err_doc = (uint32_t)(hctr[3] >> 32);
  if (err & kErrCollision) { ix->collision_doc = err_doc; return kRcCollision; }
  if (err) {
    if (err & kErrCapacity)
      return fail(TFIDF_E_CAPACITY, "vocabulary exceeds 2^%u dictionary slots (raise vocab_capacity_log2)",
                  ix->cap_log2);
    return fail(TFIDF_E_UNSUPPORTED_INPUT, "index build error flags 0x%x (doc %u)", err, err_doc);
  }
  S.doc_count = hctr[0];
  S.sum_ttf = hctr[1];
  S.nnz = hctr[2];
  S.NC = S.term_major ? 0u : (uint32_t)hctr[7];
  if (!S.term_major) HIP_TRY(S.blk.reserve((size_t)(S.n_blocks + 1) * S.NC * 4 + 16));
  // CSR tf escapes (rare: block-major only for tf >= 2^17): sorted by entry
  // index for the binary searches of the inversion and tfidf_doc_terms
  {
    const uint64_t n_esc = (uint32_t)hctr[9];
    if (n_esc > esc_cap) return fail(TFIDF_E_CAPACITY, "CSR escape list overflow");
    S.h_esc.resize(n_esc);
    if (n_esc) {
      HIP_TRY(hipMemcpyAsync(S.h_esc.data(), S.csr_esc.p, n_esc * 8, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      std::sort(S.h_esc.begin(), S.h_esc.end());
      HIP_TRY(hipMemcpyAsync(S.csr_esc.p, S.h_esc.data(), n_esc * 8, hipMemcpyHostToDevice, s));
      HIP_TRY(hipStreamSynchronize(s));
    }
  }
  if (S.nnz >= 0xFFFFFFFFull) return fail(TFIDF_E_CAPACITY, "more than 2^32 postings per shard");
  // postings: block-major u32 (post_word), term-major u64; pass-1 temp words u32
  // (term-major: the sort's u64 value buffer)
  HIP_TRY(S.post.reserve(S.nnz * (S.term_major ? 8 : 4) + 8));
  HIP_TRY(ix->post_tmp.reserve(S.nnz * (S.term_major ? 8 : 4) + 8));
  const uint64_t post_esc_cap = row_cap / kPostTfEsc + 64;       // each needs tf >= 2047 tokens of one doc
  if (!S.term_major) HIP_TRY(S.post_esc.reserve(post_esc_cap * 8));

  // the dictionary is final here (wave, Unicode and long paths done): its host
  // mirror, the deferred identity checks and the occupied-slot count run on the
  // side stream while the inversion runs (cfg-5 shape, 2^23 slots: 30.2 -> 28.4
  // ms per build; cfg 2: the 4 MB mirror, the checks and the count left ~0.2 ms
  // of copies, kernels and launch gaps after the inversion).  TFIDF_MIRROR_MAIN=1
  // keeps a mirror below 32 MB on the main stream after the inversion (A/B).
  HIP_TRY(S.h_dict.resize((size_t)2 * C));
  HIP_TRY(S.h_df.resize(C));
  // On a caller's stream (tfidf_set_stream: torch's stream under torch.distributed)
  // the small mirror stays on the main stream: the cross-stream hand-off cost the
  // one-rank RCCL rehearsal ~1 ms per step (tools/ab_dist3.sh: 12.4-12.8 vs 11.4-11.6)
  static const bool mirror_main = knob("TFIDF_MIRROR_MAIN") != nullptr;
  const bool mirror_side = (!mirror_main && s == ix->own_stream) || (size_t)2 * C * 8 >= (32u << 20);
  // (the side-stream work is enqueued after the inversion's launches, so the
  // host's enqueue time does not delay the first inversion kernel)
  if (mirror_side) HIP_TRY(hipEventRecord(ix->mir_ev[0], s));

  PostingParams pp{};
  pp.offsets = bp.offsets;
  pp.live_map = bp.live_map;
  pp.n_docs = N;
  pp.C = C;
  pp.NC = S.NC;
  pp.crank = S.crank.as<uint2>();
  pp.range_shift = S.range_shift;
  pp.n_ranges = S.R;
  pp.n_blocks = S.n_blocks;
  pp.csr = bp.csr;
  pp.csr_esc = bp.csr_esc;
  pp.n_esc = S.h_esc.size();
  pp.rsplit = bp.rsplit;
  pp.doc_norm = bp.doc_norm;
  pp.blk = S.blk.as<uint32_t>();
  pp.bbase = S.bbase.as<uint64_t>();
  pp.post = S.post.as<uint32_t>();
  pp.post_tmp = ix->post_tmp.as<uint32_t>();
  pp.post_esc = S.post_esc.as<uint64_t>();
  pp.post_esc_count = reinterpret_cast<uint32_t *>(ctr + 10);
  pp.post_esc_cap = post_esc_cap;
  pp.sort_spw = 4;
  if (const char *e = knob("TFIDF_SORT_SPW")) pp.sort_spw = (uint32_t)std::max(1, std::min(8, atoi(e)));   // A/B only (<= kSortMaxSpw)
  pp.err = bp.err;
  HIP_TRY(hipEventRecord(ix->ev[EV_D0], s));
  if (S.term_major) {
    TermParams tp{};
    if (N > kTermMaxDocs)
      return fail(TFIDF_E_CAPACITY, "the term-major layout holds at most 2^26 documents per shard");
    tp.offsets = bp.offsets;
    tp.live_map = bp.live_map;
    tp.n_docs = N;
    tp.nnz = S.nnz;
    tp.C = C;
    tp.slot_bits = ix->cap_log2;
    tp.doc_bits = 1;
    while ((1ull << tp.doc_bits) < N) tp.doc_bits++;
    // >= 4 (slot, doc <= 26 bits); at most 24 (tf <= kMaxTf): a small shard
    // (40 books: 56 - 18 - 6 = 32) must not reach a 32-bit shift in tf_esc
    tp.tf_bits = std::min(56u - tp.slot_bits - tp.doc_bits, 24u);
    if (const char *e = knob("TFIDF_TEST_TERM_TF_BITS"))      // tests: exercise the tf escape list
      tp.tf_bits = std::max(1u, std::min(tp.tf_bits, (uint32_t)atoi(e)));
    tp.csr = bp.csr;
    tp.csr_esc = bp.csr_esc;
    tp.n_esc = S.h_esc.size();
    tp.doc_nuniq = bp.doc_nuniq;
    tp.doc_norm = bp.doc_norm;
    tp.row_off = S.row_off.as<uint32_t>();
    HIP_TRY(ix->tvals.reserve(S.nnz * 8 + 16));
    tp.keys = ix->post_tmp.as<uint64_t>();
    tp.keys_alt = ix->tvals.as<uint64_t>();
    tp.post = S.post.as<uint64_t>();
    tp.toff = S.toff.as<uint64_t>();
    tp.df = S.tdf.as<uint32_t>();
    tp.err = bp.err;
    tp.tesc_cap = row_cap / ((1u << tp.tf_bits) - 1) + 64;   // each needs tf >= the escape value
    HIP_TRY(ix->term_esc.reserve(tp.tesc_cap * 16));
    tp.tesc = ix->term_esc.as<uint64_t>();
    tp.tesc_count = reinterpret_cast<uint32_t *>(ctr + 12);
    HIP_TRY(ix->term_tmp.reserve(term_invert_scratch_words(N, S.nnz, C) * 4));
    tp.scratch = ix->term_tmp.as<uint32_t>();
    // the whole inversion is reported under ms_scatter
    HIP_TRY(hipEventRecord(ix->ev[EV_DF], s));
    HIP_TRY(hipEventRecord(ix->ev[EV_BSCAN], s));
    HIP_TRY(hipEventRecord(ix->ev[EV_CSCAN], s));
    HIP_TRY(launch_term_pairs(tp, s));
    {   // tf >= 4095 (rare): the escape list sorted for the postings pass's binary search
      uint32_t ne = 0;
      HIP_TRY(hipMemcpyAsync(&ne, tp.tesc_count, 4, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      if (ne > tp.tesc_cap) return fail(TFIDF_E_CAPACITY, "term-major escape list overflow");
      if (ne) {
        std::vector<std::pair<uint64_t, uint64_t>> h(ne);
        HIP_TRY(hipMemcpy(h.data(), tp.tesc, ne * 16, hipMemcpyDeviceToHost));
        std::sort(h.begin(), h.end());
        HIP_TRY(hipMemcpy(tp.tesc, h.data(), ne * 16, hipMemcpyHostToDevice));
      }
      tp.n_tesc = ne;
    }
    HIP_TRY(launch_term_sort(tp, s));
    HIP_TRY(hipEventRecord(ix->ev[EV_SCAT], s));
  } else {
    if (S.n_blocks) {
      HIP_TRY(launch_df_partial(pp, s));
    } else {
      HIP_TRY(hipMemsetAsync(S.blk.p, 0, (size_t)S.NC * 4, s));
    }
    HIP_TRY(hipEventRecord(ix->ev[EV_DF], s));
    HIP_TRY(launch_df_sum(pp, s));
    HIP_TRY(launch_df_slots(S.crank.as<uint2>(), S.blk.as<uint32_t>() + (size_t)S.n_blocks * S.NC, C,
                            S.sdf.as<uint32_t>(), s));
    if (mirror_side) HIP_TRY(hipEventRecord(ix->mir_ev[2], s));   // df final: its host mirror copies beside the scatter
    if (S.n_blocks) HIP_TRY(launch_row_scan(pp, s));
    HIP_TRY(hipEventRecord(ix->ev[EV_BSCAN], s));
    HIP_TRY(launch_block_base(pp, s));
    HIP_TRY(hipEventRecord(ix->ev[EV_CSCAN], s));
    if (S.n_blocks) HIP_TRY(launch_scatter(pp, s));
    HIP_TRY(hipEventRecord(ix->ev[EV_SCAT], s));
  }
  if (mirror_side) {
    HIP_TRY(hipStreamWaitEvent(ix->copy_stream, ix->mir_ev[0], 0));
    HIP_TRY(hipMemcpyAsync(S.h_dict.data(), S.dict.p, (size_t)2 * C * 8, hipMemcpyDeviceToHost, ix->copy_stream));
    HIP_TRY(launch_verify_deferred(bp, ix->copy_stream));
    if (S.term_major)       // (block-major: col_rank counted the columns)
      HIP_TRY(launch_count_nonzero(S.dict.as<uint64_t>(), C, reinterpret_cast<unsigned long long *>(ctr + 7),
                                   ix->copy_stream));
    if (!S.term_major) {
      // block-major: df and the slot -> column map are final before the
      // scatter, so their host mirrors copy while it runs (on the main stream
      // after it they cost ~0.1 ms of the cfg-2 step)
      HIP_TRY(hipStreamWaitEvent(ix->copy_stream, ix->mir_ev[2], 0));
      HIP_TRY(hipMemcpyAsync(S.h_df.data(), S.df_dev(), (size_t)C * 4, hipMemcpyDeviceToHost, ix->copy_stream));
      HIP_TRY(S.h_crank.resize((size_t)C / 32 + 1));
      HIP_TRY(hipMemcpyAsync(S.h_crank.data(), S.crank.p, ((size_t)C / 32 + 1) * 8, hipMemcpyDeviceToHost,
                             ix->copy_stream));
    }
    HIP_TRY(hipEventRecord(ix->mir_ev[1], ix->copy_stream));
  }
  // host mirrors for query analysis: dictionary keys + df
  if (!mirror_side)
    HIP_TRY(hipMemcpyAsync(S.h_dict.data(), S.dict.p, (size_t)2 * C * 8, hipMemcpyDeviceToHost, s));
  if (!mirror_side || S.term_major)
    HIP_TRY(hipMemcpyAsync(S.h_df.data(), S.df_dev(), (size_t)C * 4, hipMemcpyDeviceToHost, s));
  if (!S.term_major && !mirror_side) {                 // slot -> column for query preparation
    HIP_TRY(S.h_crank.resize((size_t)C / 32 + 1));
    HIP_TRY(hipMemcpyAsync(S.h_crank.data(), S.crank.p, ((size_t)C / 32 + 1) * 8, hipMemcpyDeviceToHost, s));
  }
  if (mirror_side) {
    HIP_TRY(hipStreamWaitEvent(s, ix->mir_ev[1], 0));   // mirror, checks and count (side stream)
  } else {
    // hashed-key identity checks the tokenizers had to defer
    HIP_TRY(launch_verify_deferred(bp, s));
    // occupied dictionary slots counted on the device (ctr[7]) instead of a host
    // pass over the mirror (8 M slots at 2^23 took milliseconds)
    if (S.term_major)
      HIP_TRY(launch_count_nonzero(S.dict.as<uint64_t>(), C, reinterpret_cast<unsigned long long *>(ctr + 7), s));
  }
  uint64_t tail[8];              // ctr[3] error flags .. ctr[7] occupied slots, [8] malformed, [10] posting escapes
  HIP_TRY(hipMemcpyAsync(tail, ctr + 3, sizeof tail, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  {
    const uint64_t n_pe = S.term_major ? 0 : (uint32_t)tail[7];
    if (n_pe > post_esc_cap) return fail(TFIDF_E_CAPACITY, "posting escape list overflow");
    S.h_post_esc.resize(n_pe);
    if (n_pe) {                                // rare (tf >= 2047): sorted for the scorer's binary search
      HIP_TRY(hipMemcpy(S.h_post_esc.data(), S.post_esc.p, n_pe * 8, hipMemcpyDeviceToHost));
      std::sort(S.h_post_esc.begin(), S.h_post_esc.end());
      HIP_TRY(hipMemcpy(S.post_esc.p, S.h_post_esc.data(), n_pe * 8, hipMemcpyHostToDevice));
    }
  }
  S.malformed.resize((uint32_t)tail[5]);
  if (!S.malformed.empty()) {
    HIP_TRY(hipMemcpy(S.malformed.data(), ix->bad_list.p, S.malformed.size() * 4, hipMemcpyDeviceToHost));
    std::sort(S.malformed.begin(), S.malformed.end());
  }
  const uint32_t err2 = (uint32_t)tail[0];
  if (err2 & kErrCollision) { ix->collision_doc = (uint32_t)(tail[0] >> 32); return kRcCollision; }
  if (err2 & kErrTfTooLarge) return fail(TFIDF_E_UNSUPPORTED_INPUT, "a term frequency exceeds 2^24 - 1");
  S.num_terms = tail[4];

  tfidf_commit_timing &t = ix->timing;
  t.ms_tokenize = ev_ms(ix, EV_START, EV_TOK);
  t.ms_long = n_long ? ev_ms(ix, EV_L0, EV_LONG) : 0.0f;
  t.ms_df = ev_ms(ix, EV_D0, EV_DF);
  t.ms_blockscan = ev_ms(ix, EV_DF, EV_BSCAN);
  t.ms_colscan = ev_ms(ix, EV_BSCAN, EV_CSCAN);
  t.ms_scatter = ev_ms(ix, EV_CSCAN, EV_SCAT);
  t.ms_total = t.ms_tokenize + t.ms_long + ev_ms(ix, EV_D0, EV_SCAT);   // device time, host syncs excluded
  t.text_bytes = ix->text_bytes;
  t.num_docs = N;
  t.nnz = S.nnz;

  // what the snapshot was built from
  S.cap_log2 = ix->cap_log2;
  S.text_bytes = ix->text_bytes;
  S.text = ix->text;
  S.offsets = ix->offsets;
  ix->keys.compact();
  S.keys = ix->keys;                 // shares the chunks; the builder appends to a new one
  S.hash_seed = ix->hash_seed;
  {
    std::lock_guard<std::mutex> tl(S.term_mu);
    S.term_cache.clear();
  }
  // statistics in force: the shard's own (a GLOBAL exchange publishes another view)
  if (!S.stats || S.stats.use_count() > 1) S.stats = std::make_shared<StatsView>(ix->cfg.device);
  StatsView &V = *S.stats;
  if (int rc = V.wait_gdf()) return rc;
  V.global = false;
  V.gdf.clear();
  V.doc_count = S.doc_count;
  V.sum_ttf = S.sum_ttf;
  return upload_cache(ix->cfg, V, s);
}

extern "C" int tfidf_commit(tfidf_index *ix) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard g(ix->cfg.device);
  // The build target: the previous snapshot if no search holds it any more
  // (its buffers are reused as they are), else a new one.  The published
  // snapshot stays searchable until this build succeeds; a failed build
  // publishes nothing (the reference's readers keep the last commit).
  std::shared_ptr<Snapshot> S;
  if (ix->spare && ix->spare.use_count() == 1) S = std::move(ix->spare);
  ix->spare.reset();
  if (!S) S = std::make_shared<Snapshot>(ix->cfg.device);
  // Hash seeds: 0, then 1, 2, 3 after a detected collision (TFIDF_TEST_WEAK_HASH:
  // start from a seed under which equal-length hashed keys collide).  A floor
  // set by tfidf_set_hash_attempt (GLOBAL statistics: every shard must hash
  // with one seed) skips the earlier attempts.
  const char *weak = knob("TFIDF_TEST_WEAK_HASH");
  ix->hash_seed = ix->hash_floor ? ix->hash_floor : ((weak && atoi(weak)) ? kWeakHashSeed : 0);
  ix->hash_rebuilds = ix->hash_floor;
  for (uint32_t attempt = ix->hash_floor;; attempt++) {
    int rc = commit_once(ix, *S);
    if (rc != TFIDF_OK) {
      hipStreamSynchronize(ix->stream);        // nothing of this build may still run on either stream
      hipStreamSynchronize(ix->copy_stream);
    }
    if (rc == kRcCollision) {
      if (attempt == 3) {
        ix->spare = std::move(S);
        return fail(TFIDF_E_UNSUPPORTED_INPUT, "hash collisions under 4 seeds (last in document %u)", ix->collision_doc);
      }
      ix->hash_seed = attempt + 1;
      ix->hash_rebuilds++;
      continue;
    }
    if (rc != TFIDF_OK) {
      ix->spare = std::move(S);
      return rc == kRcNoPublish ? TFIDF_OK : rc;
    }
    S->hash_rebuilds = ix->hash_rebuilds;
    S->generation = ++ix->generation;
    {
      std::lock_guard<std::mutex> sl(ix->snap_mu);
      std::swap(ix->cur, S);                   // published; S = the previous snapshot
    }
    ix->spare = std::move(S);                  // rebuilt in place next time if no search holds it
    return TFIDF_OK;
  }
}

extern "C" int tfidf_set_hash_attempt(tfidf_index *ix, uint32_t attempt) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL index");
  if (attempt > 3) return fail(TFIDF_E_INVALID_ARG, "hash seed attempt %u > 3", attempt);
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->hash_floor = attempt;
  return TFIDF_OK;
}

extern "C" int tfidf_get_commit_timing(const tfidf_index *ix, tfidf_commit_timing *out) {
  if (!ix || !out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  *out = ix->timing;
  return TFIDF_OK;
}

extern "C" int tfidf_stats(const tfidf_index *ix, tfidf_index_stats *out) {
  if (!ix || !out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  const std::shared_ptr<Snapshot> S = current(ix);
  *out = tfidf_index_stats{};
  uint64_t staged_bytes = 0;
  {
    // builder-side fields: add_docs / clear / commit replace them under mu
    std::lock_guard<std::mutex> lk(const_cast<tfidf_index *>(ix)->mu);
    out->text_bytes = ix->text_bytes;
    out->hash_seed = ix->hash_seed;
    out->hash_rebuilds = ix->hash_rebuilds;
    staged_bytes = ix->text->bytes + ix->offsets->bytes;
  }
  if (S) {
    out->num_docs = S->n_docs;
    out->doc_count = S->doc_count;
    out->sum_ttf = S->sum_ttf;
    out->num_terms = S->num_terms;
    out->nnz = S->nnz;
    out->long_docs = S->long_docs;
    out->term_major = S->term_major;
    out->pack_docs = S->pack_docs;
    out->pack_retried = S->pack_retried;
    out->unicode_docs = S->unicode_docs;
    out->unicode_wave_docs = S->unicode_wave_docs;
    out->long_chunked = S->long_chunked;
    out->malformed_docs = S->malformed.size();
    out->hash_seed = S->hash_seed;
    out->hash_rebuilds = S->hash_rebuilds;
  }
  {
    std::lock_guard<std::mutex> cl(ix->cq_mu);
    out->coalesced_batches = ix->cq_batches;
    out->coalesced_queries = ix->cq_queries;
  }
  out->unit_batches = ix->unit_batches.load();
  out->fused_queries = ix->fused_queries.load();
  out->unit_count = ix->unit_count.load();
  uint64_t tot = staged_bytes;
  if (S) {
    const DevBuf *bufs[] = {&S->dict, &S->csr, &S->csr_esc, &S->doc_len, &S->doc_nuniq, &S->doc_norm,
                            &S->rsplit, &S->blk, &S->bbase, &S->post, &S->toff, &S->tdf, &S->crank, &S->sdf};
    for (const DevBuf *b : bufs) tot += b->bytes;
  }
  out->device_bytes = tot;
  return TFIDF_OK;
}

// ---------------------------------------------------------------------------
// dictionary (host mirror)

static uint32_t host_lookup(const Snapshot &S, uint64_t lo, uint64_t hi) {
  if (S.C == 0) return kInvalidSlot;
  const uint32_t mask = S.C - 1;
  // same probe order as the device (kernels_index.hip dict_lookup_multi):
  // linear from the aligned 2-slot bucket of the hash; lo[C] then hi[C]
  uint32_t s = dict_home(dict_hash(lo, hi), mask) & ~1u;
  for (uint32_t it = 0; it <= mask; it++) {
    const uint64_t clo = S.h_dict[s], chi = S.h_dict[(size_t)S.C + s];
    if (clo == 0) return kInvalidSlot;
    if (clo == lo && chi == hi) return s;
    s = (s + 1) & mask;
  }
  return kInvalidSlot;
}

// Lower-cased term string of dictionary slot `slot`: decoded from an exact
// key, or (hashed key) read from its reference occurrence in the corpus.
struct StrSink {
  std::string s;
  void push(uint8_t c) { s.push_back((char)c); }
};
static int slot_term(Snapshot &S, uint32_t slot, std::string *out) {
  char b[32];
  const uint64_t lo = S.h_dict[slot], hi = S.h_dict[(size_t)S.C + slot];
  if (const uint32_t n = key_decode(lo, hi, b)) { out->assign(b, n); return TFIDF_OK; }
  std::lock_guard<std::mutex> tl(S.term_mu);             // batch preparation threads share the cache
  auto it = S.term_cache.find(slot);
  if (it != S.term_cache.end()) { *out = it->second; return TFIDF_OK; }
  uint64_t r = 0;
  HIP_TRY(hipMemcpy(&r, S.dict.as<uint64_t>() + 2 * (size_t)S.C + slot, 8, hipMemcpyDeviceToHost));
  if (r == 0) return fail(TFIDF_E_STATE, "dictionary slot %u has no reference occurrence", slot);
  std::vector<uint8_t> raw(dict_ref_len(r));
  if (!raw.empty())
    HIP_TRY(hipMemcpy(raw.data(), S.text->as<uint8_t>() + dict_ref_off(r), raw.size(), hipMemcpyDeviceToHost));
  StrSink sink;
  uc_token_bytes(raw.data(), raw.size(), 0, raw.size(), sink);
  S.term_cache.emplace(slot, sink.s);
  *out = sink.s;
  return TFIDF_OK;
}

// Dictionary slot of the (lower-cased) term t, kInvalidSlot if absent; a
// hashed key must also match the slot's term string.
static uint32_t lookup_term(Snapshot &S, const std::string &t) {
  uint64_t lo, hi;
  term_key(t, &lo, &hi, S.hash_seed);
  const uint32_t s = host_lookup(S, lo, hi);
  if (s == kInvalidSlot || !key_is_hashed(lo)) return s;
  std::string ts;
  if (slot_term(S, s, &ts) != TFIDF_OK || ts != t) return kInvalidSlot;
  return s;
}

struct PreparedQuery {
  std::vector<uint32_t> slot;    // per term: what the scorers index it by (Snapshot::col_of)
  std::vector<uint32_t> ldf;     // per term: the shard's own df
  std::vector<float> w;
  std::vector<uint32_t> role;    // role << 24 | MUST clause index
  uint32_t meta = 0;             // MUST clause count | has MUST_NOT << 31
};

// upper bound of a query's hits on this shard: the sum of its scoring terms' local df
static uint64_t hits_bound(const Snapshot &S, const PreparedQuery &pq) {
  uint64_t b = 0;
  for (size_t i = 0; i < pq.slot.size(); i++)
    if ((pq.role[i] >> 24) != kRoleNot) b += pq.ldf[i];
  return b;
}

// Query plan (analysis.h) -> dictionary slots + BM25 weights.  A term absent
// from this shard's dictionary has no scorer (TermWeight.scorer == null): a
// SHOULD or MUST_NOT term is dropped, a MUST clause without any present term
// leaves the query without hits (BooleanWeight: required scorer missing), and
// a query with neither MUST clauses nor a present SHOULD term has no hits.
static int prepare_query(Snapshot &S, StatsView &V, const uint8_t *q, uint64_t n, PreparedQuery *pq) {
  QueryPlan plan;
  const int rc = parse_query(q, n, &plan);
  if (rc == kQBadUtf8) return fail(TFIDF_E_UNSUPPORTED_QUERY, "query is not valid UTF-8");
  if (rc == kQSyntax)
    return fail(TFIDF_E_QUERY_SYNTAX, "query does not parse (QueryParser ParseException / TooManyClauses)");
  if (int e = V.wait_gdf()) return e;
  const uint64_t dc = V.doc_count;
  if (dc == 0) return TFIDF_OK;                        // no document holds a token
  std::vector<uint32_t> present(plan.n_groups, 0);
  uint32_t n_should = 0;
  bool has_not = false;
  for (const PlanTerm &t : plan.terms) {
    const uint32_t s = lookup_term(S, t.term);
    if (s == kInvalidSlot) continue;                   // absent term contributes nothing
    float wv = 0.0f;
    if (t.role != kRoleNot) {
      const uint64_t df = V.global ? V.gdf[s] : S.h_df[s];
      const float idf = bm25_idf(df, dc);
      volatile float w = t.boost * idf;                // BM25Scorer: weight = boost * idf
      wv = w;
    }
    if (t.role == kRoleMust) present[t.group]++;
    if (t.role == kRoleShould) n_should++;
    if (t.role == kRoleNot) has_not = true;
    pq->slot.push_back(S.col_of(s));
    pq->ldf.push_back(S.h_df[s]);
    pq->w.push_back(wv);
    pq->role.push_back(t.role << 24 | t.group);
  }
  bool empty = plan.n_groups == 0 && n_should == 0;
  for (uint32_t c : present) empty |= c == 0;
  if (empty) {
    pq->slot.clear();
    pq->ldf.clear();
    pq->w.clear();
    pq->role.clear();
    return TFIDF_OK;
  }
  pq->meta = plan.n_groups | (has_not ? 1u << 31 : 0u);
  return TFIDF_OK;
}

// Batch of prepared queries in device layout.
struct QueryBatch {
  std::vector<uint32_t> off{0}, slot, role, meta, ldf;
  std::vector<float> w;
  bool ops = false;                // some query has MUST / MUST_NOT clauses
  void add(const PreparedQuery &pq) {
    slot.insert(slot.end(), pq.slot.begin(), pq.slot.end());
    ldf.insert(ldf.end(), pq.ldf.begin(), pq.ldf.end());
    w.insert(w.end(), pq.w.begin(), pq.w.end());
    role.insert(role.end(), pq.role.begin(), pq.role.end());
    off.push_back((uint32_t)slot.size());
    meta.push_back(pq.slot.empty() ? 0u : pq.meta);
    ops |= !pq.slot.empty() && pq.meta != 0;
  }
};

// Prepare a batch's queries (parse, analysis, dictionary lookups, BM25
// weights) on host threads: large batches spend more time here than on the
// device (10 k queries: ~10 ms on one thread).  A query that does not parse
// (or is not UTF-8) has no hits, as the reference answers [] for it
// (Worker.java:182-185); the batch goes on.
// Persistent host workers for batch query preparation (spawning 16 threads per
// batch cost ~0.5 ms of a 10 k-query batch).  run(n, fn): fn(a, b) over `parts`
// slices of [0, n), the caller taking slice 0; one batch at a time.
struct PrepPool {
  std::vector<std::thread> th;
  std::mutex run_mu, mu;
  std::condition_variable cv, done_cv;
  std::function<void(uint32_t, uint32_t)> fn;
  uint32_t n = 0, parts = 0, next = 0, finished = 0;
  uint64_t gen = 0;
  explicit PrepPool(uint32_t workers) {
    for (uint32_t i = 0; i < workers; i++) th.emplace_back([this] { loop(); });
  }
  void slice(uint32_t i) { fn((uint32_t)((uint64_t)n * i / parts), (uint32_t)((uint64_t)n * (i + 1) / parts)); }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return gen != seen; });
      seen = gen;
      while (next < parts) {
        const uint32_t i = next++;
        lk.unlock();
        slice(i);
        lk.lock();
        if (++finished == parts) done_cv.notify_all();
      }
    }
  }
  void run(uint32_t n_items, uint32_t n_parts, std::function<void(uint32_t, uint32_t)> f) {
    std::lock_guard<std::mutex> rl(run_mu);
    std::unique_lock<std::mutex> lk(mu);
    fn = std::move(f);
    n = n_items;
    parts = n_parts;
    next = 1;                                           // slice 0: the caller
    finished = 0;
    gen++;
    cv.notify_all();
    lk.unlock();
    slice(0);
    lk.lock();
    if (++finished < parts) done_cv.wait(lk, [&] { return finished == parts; });
  }
};
static PrepPool *prep_pool() {
  // never destroyed: its threads block forever on an idle pool
  static PrepPool *pool = new PrepPool(std::min<uint32_t>(std::max(1u, std::thread::hardware_concurrency()), 16u) - 1);
  return pool;
}

static int prepare_batch(tfidf_index *ix, Snapshot &S, StatsView &V, const uint8_t *q_utf8,
                         const uint64_t *q_offsets, uint32_t n_q, QueryBatch *qb) {
  if (int e = V.wait_gdf()) return e;                  // once, before the workers read the mirrors
  std::vector<PreparedQuery> pqs(n_q);
  auto work = [&](uint32_t a, uint32_t b) {
    DeviceGuard g(ix->cfg.device);                      // slot_term may read a reference occurrence
    for (uint32_t i = a; i < b; i++)
      if (prepare_query(S, V, q_utf8 + q_offsets[i], q_offsets[i + 1] - q_offsets[i], &pqs[i]) != TFIDF_OK)
        pqs[i] = PreparedQuery();
  };
  uint32_t nt = std::min<uint32_t>(std::max(1u, std::thread::hardware_concurrency()), 16u);
  nt = std::max(1u, std::min(nt, n_q / 128));
  if (nt <= 1) work(0, n_q);
  else prep_pool()->run(n_q, nt, work);
  size_t ns = 0;
  for (const PreparedQuery &pq : pqs) ns += pq.slot.size();
  qb->slot.reserve(ns);
  qb->ldf.reserve(ns);
  qb->w.reserve(ns);
  qb->role.reserve(ns);
  qb->off.reserve(n_q + 1);
  qb->meta.reserve(n_q);
  for (const PreparedQuery &pq : pqs) qb->add(pq);
  return TFIDF_OK;
}

// Test hook (TFIDF_TEST_FAIL_SCORING = n): every n-th scoring call fails after
// its kernels are queued, as a HIP error in a later launch would
// (tests/test_gpu_snapshot.py: the failed search must drain before its
// snapshot can be rebuilt by a commit).
static int scoring_done() {
  const char *e = knob("TFIDF_TEST_FAIL_SCORING");
  if (!e) return TFIDF_OK;
  static std::atomic<uint64_t> calls{0};
  const uint64_t n = (uint64_t)std::max(1, atoi(e));
  if (++calls % n) return TFIDF_OK;
  return fail(TFIDF_E_HIP, "injected scoring failure (TFIDF_TEST_FAIL_SCORING)");
}

static int run_scoring(tfidf_index *ix, Snapshot &S, StatsView &V, SearchCtx &X, hipStream_t s, const QueryBatch &qb,
                       uint32_t n_q, uint32_t k) {
  const std::vector<uint32_t> &qoff = qb.off, &slots = qb.slot;
  const size_t ns = slots.size(), nr = qb.ops ? ns + qb.meta.size() : 0;
  const size_t npairs = (size_t)n_q * S.n_blocks;
  const bool batch = k && npairs >= (size_t)ix->num_cus * 16 && npairs < (1ull << 32);
  // batches of plain disjunctions, k <= 64, block-major: workgroup per
  // (query, block range) unit (k_score_units); units of about unit_post
  // postings, queries above that split into equal block ranges, listed first
  // (heavy units start early, the light tail balances)
  std::vector<uint32_t> &units = X.q_units;
  units.clear();
  bool unit_path = batch && k <= kUnitMaxK && !qb.ops && !S.term_major && !knob("TFIDF_NO_UNITS");
  uint32_t n_wunits = 0;                 // the first n_wunits units are wave units
  if (unit_path) {
    std::vector<uint64_t> P(n_q, 0);
    uint64_t T = 0;
    for (uint32_t q = 0; q < n_q && unit_path; q++) {
      if (qoff[q + 1] - qoff[q] > kUnitMaxTerms) unit_path = false;
      for (uint32_t t = qoff[q]; t < qoff[q + 1]; t++)
        if (slots[t] != kInvalidSlot) P[q] += qb.ldf[t];
      T += P[q];
    }
    // light queries (at most light_post postings per block on average): wave
    // units (k_score_wunits, units of ~16 k postings); heavy ones: workgroup
    // units (k_score_units, dense block accumulator; ~T/4096 postings each)
    const uint32_t nb = S.n_blocks;
    uint64_t light_post = kWunitLightPost;
    if (const char *e = knob("TFIDF_WUNIT_LIGHT")) light_post = (uint64_t)atoll(e);   // A/B and test hook
    uint64_t unit_post = std::min<uint64_t>(std::max<uint64_t>(T / 4096, 8192), 1ull << 17);
    uint64_t wunit_post = 16384;
    if (const char *e = knob("TFIDF_UNIT_POST")) unit_post = wunit_post = std::max(1, atoi(e));   // test hook: force splits
    for (int pass = 0; pass < 3 && unit_path; pass++)        // light; heavy split; heavy whole
      for (uint32_t q = 0; q < n_q; q++) {
        const bool light = P[q] <= light_post * nb;
        if (light != (pass == 0)) continue;
        const uint64_t up = light ? wunit_post : unit_post;
        const uint64_t nch = std::min<uint64_t>(std::max<uint64_t>((P[q] + up - 1) / up, 1), nb);
        if (!light && (nch > 1) != (pass == 1)) continue;
        for (uint64_t c = 0; c < nch; c++) {
          units.push_back(q);
          units.push_back((uint32_t)(c * nb / nch));
          units.push_back((uint32_t)((c + 1) * nb / nch));
          units.push_back(0);
        }
        if (light) n_wunits += (uint32_t)nch;
      }
    if (!unit_path) units.clear();
  }
  const size_t words0 = (qoff.size() + 2 * ns + nr + 3) & ~(size_t)3;    // units 16-B aligned
  const size_t words = words0 + units.size();
  // one pinned staging buffer, one upload (the previous upload out of it must
  // have left: batch searches return before their copies run)
  if (X.q_in_pending) HIP_TRY(hipEventSynchronize(X.q_in_ev));
  HIP_TRY(X.q_host.resize(words));
  uint32_t *h = X.q_host.data();
  memcpy(h, qoff.data(), qoff.size() * 4);
  memcpy(h + qoff.size(), slots.data(), ns * 4);
  memcpy(h + qoff.size() + ns, qb.w.data(), ns * 4);
  if (qb.ops) {
    memcpy(h + qoff.size() + 2 * ns, qb.role.data(), ns * 4);
    memcpy(h + qoff.size() + 3 * ns, qb.meta.data(), qb.meta.size() * 4);
  }
  if (!units.empty()) memcpy(h + words0, units.data(), units.size() * 4);
  if (words * 4 + 16 > X.q_in.bytes) {
    // a pending chunk of a pipelined batch may still read q_in: finish it
    // before the buffer is replaced (1.5x headroom, so later chunks rarely grow it)
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(X.q_in.reserve(words * 6 + 16));
  }
  HIP_TRY(hipMemcpyAsync(X.q_in.p, h, words * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipEventRecord(X.q_in_ev, s));
  X.q_in_pending = true;
  uint32_t *din = X.q_in.as<uint32_t>();
  QueryParams qp{};
  qp.post = S.post.as<uint64_t>();
  qp.post32 = S.post.as<uint32_t>();
  qp.post_esc = S.post_esc.as<uint64_t>();
  qp.n_post_esc = S.h_post_esc.size();
  qp.bbase = S.bbase.as<uint64_t>();
  qp.blk = S.blk.as<uint32_t>();
  qp.toff = S.term_major ? S.toff.as<uint64_t>() : nullptr;
  qp.C = S.qcols();
  qp.n_blocks = S.n_blocks;
  qp.n_docs = S.n_docs;
  qp.cache = V.cache.as<float>();
  qp.q_off = din;
  qp.q_slot = din + qoff.size();
  qp.q_w = reinterpret_cast<const float *>(din + qoff.size() + ns);
  qp.q_role = qb.ops ? din + qoff.size() + 2 * ns : nullptr;
  qp.q_meta = qb.ops ? din + qoff.size() + 3 * ns : nullptr;
  qp.ops = qb.ops ? 1u : 0u;
  qp.n_q = n_q;
  qp.k = k;
  {   // enough (block, chunk) workgroups to fill the chip ~4 deep; never more chunks than queries
    const uint32_t want = (uint32_t)ix->num_cus * 4;
    uint32_t chunks = S.n_blocks ? (want + S.n_blocks - 1) / S.n_blocks : 1;
    chunks = std::max(1u, std::min(chunks, n_q));
    qp.q_chunk = (n_q + chunks - 1) / chunks;
  }
  if (k) {
    HIP_TRY(X.cand.reserve((size_t)n_q * S.n_blocks * k * 8 + 8));
    HIP_TRY(X.cand_n.reserve((size_t)n_q * S.n_blocks * 4 + 4));
    // results contiguous (doc | score | n): a single query reads them back in one copy
    HIP_TRY(X.q_out.reserve(((size_t)2 * n_q * k + n_q) * 4 + 16));
    X.res_doc = X.q_out.as<uint32_t>();
    X.res_score = reinterpret_cast<float *>(X.res_doc + (size_t)n_q * k);
    X.res_n = X.res_doc + (size_t)2 * n_q * k;
    qp.cand = X.cand.as<uint64_t>();
    qp.cand_n = X.cand_n.as<uint32_t>();
    qp.out_doc = X.res_doc;
    qp.out_score = X.res_score;
    qp.out_n = X.res_n;
  } else {
    HIP_TRY(X.hits.reserve((size_t)S.n_blocks * kBlockDocs * 8 + 8));
    HIP_TRY(X.hits_n.reserve((size_t)S.n_blocks * 4 + 4));
    qp.hits = X.hits.as<uint64_t>();
    qp.hits_n = X.hits_n.as<uint32_t>();
  }
  if (X.q_timing && X.q_rec_start) HIP_TRY(hipEventRecord(X.ev[QEV_0], s));
  if (unit_path) {
    HIP_TRY(X.ovf.reserve(64));
    uint32_t *ctr = X.ovf.as<uint32_t>();
    HIP_TRY(hipMemsetAsync(ctr, 0, 8, s));
    const uint32_t n_units = (uint32_t)(units.size() / 4), n_gunits = n_units - n_wunits;
    ix->unit_batches++;
    ix->unit_count += n_units;
    const uint4 *ud = reinterpret_cast<const uint4 *>(din + words0);
    // both kinds at once: the wave units on the side stream (fork / join events),
    // so the two latency-bound kernels share the CUs instead of running in turn
    const bool both = n_wunits && n_gunits;
    hipStream_t ws = both ? X.side : s;
    if (both) {
      HIP_TRY(hipEventRecord(X.q_ev[0], s));
      HIP_TRY(hipStreamWaitEvent(ws, X.q_ev[0], 0));
    }
    if (n_wunits) {
      uint32_t wper_cu = kWunitWGsPerCU;
      if (const char *e = knob("TFIDF_WUNIT_WG_PER_CU")) wper_cu = (uint32_t)std::max(1, atoi(e));   // A/B
      const int grid = (int)std::min<uint64_t>((n_wunits + kWunitWavesPerWG - 1) / kWunitWavesPerWG,
                                               (uint64_t)ix->num_cus * wper_cu);
      HIP_TRY(launch_score_wunits(qp, ud, n_wunits, ctr, grid, ws));
    }
    if (n_gunits) {
      // (one per CU next to the wave units measured slower: 6.3 -> 7.8 ms at cfg 4)
      uint32_t per_cu = kUnitWGsPerCU;
      if (const char *e = knob("TFIDF_UNIT_WG_PER_CU")) per_cu = (uint32_t)std::max(1, atoi(e));   // A/B
      const int grid = (int)std::min<uint64_t>(n_gunits, (uint64_t)ix->num_cus * per_cu);
      HIP_TRY(launch_score_units(qp, ud + n_wunits, n_gunits, ctr + 1, grid, s));
    }
    if (both) {
      HIP_TRY(hipEventRecord(X.q_ev[1], ws));
      HIP_TRY(hipStreamWaitEvent(s, X.q_ev[1], 0));
    }
    if (X.q_timing) HIP_TRY(hipEventRecord(X.ev[QEV_1], s));
    HIP_TRY(launch_merge_topk(qp, s));
    if (X.q_timing) HIP_TRY(hipEventRecord(X.ev[QEV_2], s));
    return scoring_done();
  }
  if (batch) {
    // batches: wave per (block, query) pair; pairs with many postings are
    // listed for the dense per-block kernel (list mode, persistent grid).
    // Single queries keep the dense kernel: a few hundred pairs cannot fill
    // the chip one wave each.
    // plain heavy pairs -> ovf list (k_score_blocks<false>); pairs of operator
    // queries -> ovf2 list (k_score_blocks<true>)
    HIP_TRY(X.ovf.reserve(npairs * 8 + 64));
    qp.ovf_count = X.ovf.as<uint32_t>();
    qp.ovf2_count = qp.ovf_count + 1;
    qp.ovf_list = qp.ovf_count + 16;
    qp.ovf2_list = qp.ovf_list + npairs;
    qp.list_grid = (uint32_t)ix->num_cus * 2;
    HIP_TRY(hipMemsetAsync(qp.ovf_count, 0, 8, s));
    const uint64_t want = (npairs + kPairWavesPerWG - 1) / kPairWavesPerWG;
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)ix->num_cus * 40));
    HIP_TRY(launch_score_pairs(qp, grid, s));
    qp.ops = 0;
    if (qb.ops) {
      QueryParams q2 = qp;
      q2.ovf_list = qp.ovf2_list;
      q2.ovf_count = qp.ovf2_count;
      q2.ops = 1;
      q2.list_grid = (uint32_t)ix->num_cus;          // one 134 KiB workgroup per CU
      HIP_TRY(launch_score_blocks(q2, s));
    }
  }
  HIP_TRY(launch_score_blocks(qp, s));
  if (X.q_timing) HIP_TRY(hipEventRecord(X.ev[QEV_1], s));
  if (k) HIP_TRY(launch_merge_topk(qp, s));
  if (X.q_timing) HIP_TRY(hipEventRecord(X.ev[QEV_2], s));
  return scoring_done();
}

// One search on a snapshot (tfidf_search: the published one; tfidf_reader_search:
// the reader's).
static int search_on(tfidf_index *ix, Snapshot &S, StatsView &V, const uint8_t *q, uint64_t q_len, uint32_t k,
                     uint32_t *doc_ids, float *scores, uint64_t cap, uint64_t *n_out) {
  CtxLease lease(ix);
  if (lease.rc) return lease.rc;
  SearchCtx &X = *lease.c;
  const hipStream_t s = lease.stream();
  if (k > 1024) return fail(TFIDF_E_INVALID_ARG, "k must be <= 1024 (0 = all hits)");
  DeviceGuard g(ix->cfg.device);
  PreparedQuery pq;
  int rc = prepare_query(S, V, q, q_len, &pq);
  if (rc) return rc;
  if (pq.slot.empty() || S.n_docs == 0) { set_last_ms(ix, 0, 0); return TFIDF_OK; }
  // fused path for k <= kFusedMaxK: each block workgroup writes its k
  // candidates to pinned host memory over PCIe and the host merges n_blocks x k
  // keys, a cost that grows with k (larger k: run_scoring + the device merge)
  if (k && k <= kFusedMaxK && pq.slot.size() <= kInlTerms && !knob("TFIDF_NO_FUSED")) {
    // one launch: query terms in the kernel arguments, block scoring with the
    // candidates written to pinned host memory, merged here
    HIP_TRY(X.q_res.resize((size_t)2 * k + 1));
    QueryParams qp{};
    qp.post = S.post.as<uint64_t>();
    qp.post32 = S.post.as<uint32_t>();
    qp.post_esc = S.post_esc.as<uint64_t>();
    qp.n_post_esc = S.h_post_esc.size();
    qp.bbase = S.bbase.as<uint64_t>();
    qp.blk = S.blk.as<uint32_t>();
    qp.toff = S.term_major ? S.toff.as<uint64_t>() : nullptr;
    qp.C = S.qcols();
    qp.n_blocks = S.n_blocks;
    qp.n_docs = S.n_docs;
    qp.cache = V.cache.as<float>();
    qp.inl_n = (uint32_t)pq.slot.size();
    qp.inl_meta = pq.meta;
    for (size_t i = 0; i < pq.slot.size(); i++) {
      qp.inl_slot[i] = pq.slot[i];
      qp.inl_w[i] = pq.w[i];
      qp.inl_role[i] = pq.role[i];
    }
    qp.ops = pq.meta != 0 ? 1u : 0u;
    qp.n_q = 1;
    qp.q_chunk = 1;
    qp.k = k;
    // the block workgroups write their candidates to pinned host memory; the
    // host merges them (a merge kernel + copies: p50 0.049 / 0.057 ms, this
    // path 0.034 ms; a last-workgroup merge in the scoring kernel 0.055 ms:
    // its device-scope fences cost more than the launch they save)
    HIP_TRY(X.q_cand_h.resize((size_t)S.n_blocks * k * 2 + S.n_blocks));
    qp.cand = reinterpret_cast<uint64_t *>(X.q_cand_h.data());
    qp.cand_n = X.q_cand_h.data() + (size_t)S.n_blocks * k * 2;
    if (X.q_timing) HIP_TRY(hipEventRecord(X.ev[QEV_0], s));
    HIP_TRY(launch_score_blocks(qp, s));
    if (X.q_timing) {
      HIP_TRY(hipEventRecord(X.ev[QEV_1], s));
      HIP_TRY(hipEventRecord(X.ev[QEV_2], s));
    }
    ix->fused_queries++;
    HIP_TRY(hipStreamSynchronize(s));
    {
      // the blocks' candidate keys (score bits << 32 | ~doc: unique, key order =
      // score desc, doc asc) -> top k
      const uint64_t *ck = reinterpret_cast<const uint64_t *>(X.q_cand_h.data());
      const uint32_t *cn = X.q_cand_h.data() + (size_t)S.n_blocks * k * 2;
      std::vector<uint64_t> &all = X.q_merge;
      all.clear();
      for (uint32_t b = 0; b < S.n_blocks; b++)
        for (uint32_t i = 0; i < cn[b]; i++) all.push_back(ck[(size_t)b * k + i]);
      const size_t m = std::min<size_t>(k, all.size());
      std::partial_sort(all.begin(), all.begin() + m, all.end(), std::greater<uint64_t>());
      uint32_t *h = X.q_res.data();
      for (size_t i = 0; i < m; i++) {
        h[i] = ~(uint32_t)all[i];
        uint32_t sb = (uint32_t)(all[i] >> 32);
        memcpy(&h[k + i], &sb, 4);
      }
      h[2 * k] = (uint32_t)m;
    }
    const uint32_t n = X.q_res[2 * k];
    *n_out = n;
    if (n > cap) return fail(TFIDF_E_BUFFER, "need %u result slots", n);
    memcpy(doc_ids, X.q_res.data(), n * 4);
    memcpy(scores, X.q_res.data() + k, n * 4);
    set_last_ms(ix, qev_ms(X, QEV_0, QEV_1), qev_ms(X, QEV_0, QEV_2));
    return TFIDF_OK;
  }
  QueryBatch qb;
  qb.add(pq);
  rc = run_scoring(ix, S, V, X, s, qb, 1, k);
  if (rc) return rc;
  if (k) {
    // one copy of (doc[k] | score[k] | n) into pinned memory, one wait
    HIP_TRY(X.q_res.resize((size_t)2 * k + 1));
    HIP_TRY(hipMemcpyAsync(X.q_res.data(), X.res_doc, ((size_t)2 * k + 1) * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    X.q_in_pending = false;
    const uint32_t n = X.q_res[2 * k];
    *n_out = n;
    if (n > cap) return fail(TFIDF_E_BUFFER, "need %u result slots", n);
    memcpy(doc_ids, X.q_res.data(), n * 4);
    memcpy(scores, X.q_res.data() + k, n * 4);
    set_last_ms(ix, qev_ms(X, QEV_0, QEV_1), qev_ms(X, QEV_0, QEV_2));
    return TFIDF_OK;
  }
  // all hits: per-block sorted runs -> merge passes on the device -> (doc, score)
  const uint32_t R = S.n_blocks;
  HIP_TRY(X.hits_c.reserve((size_t)R * kBlockDocs * 8 + 8));
  HIP_TRY(X.hits_s.reserve((size_t)R * kBlockDocs * 8 + 8));
  HIP_TRY(X.hits_P.reserve(((size_t)R + 1) * 8));
  HIP_TRY(X.out_doc.reserve((size_t)R * kBlockDocs * 4 + 4));
  HIP_TRY(X.out_score.reserve((size_t)R * kBlockDocs * 4 + 4));
  HIP_TRY(launch_hits_order(X.hits.as<uint64_t>(), X.hits_n.as<uint32_t>(), R, X.hits_P.as<uint64_t>(),
                            X.hits_c.as<uint64_t>(), X.hits.as<uint64_t>(), X.hits_s.as<uint64_t>(),
                            X.out_doc.as<uint32_t>(),
                            X.out_score.as<float>(), nullptr, 0, hits_bound(S, pq), ix->num_cus * 4, s));
  if (X.q_timing) HIP_TRY(hipEventRecord(X.ev[QEV_2], s));
  uint64_t H = 0;
  HIP_TRY(hipMemcpyAsync(&H, X.hits_P.as<uint64_t>() + R, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  *n_out = H;
  if (H > cap) return fail(TFIDF_E_BUFFER, "need %llu result slots", (unsigned long long)H);
  if (H) {
    HIP_TRY(hipMemcpyAsync(doc_ids, X.out_doc.p, H * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(scores, X.out_score.p, H * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  set_last_ms(ix, qev_ms(X, QEV_0, QEV_1), qev_ms(X, QEV_0, QEV_2));
  return TFIDF_OK;
}

extern "C" int tfidf_search(tfidf_index *ix, const uint8_t *q, uint64_t q_len, uint32_t k, uint32_t *doc_ids,
                            float *scores, uint64_t cap, uint64_t *n_out) {
  if (!ix || (!q && q_len) || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  *n_out = 0;
  std::shared_ptr<StatsView> view;
  const std::shared_ptr<Snapshot> snap = current(ix, &view);
  if (!snap) return fail(TFIDF_E_STATE, "search before commit");
  return search_on(ix, *snap, *view, q, q_len, k, doc_ids, scores, cap, n_out);
}

static int doc_keys_of(const Snapshot *S, uint8_t *buf, uint64_t cap, uint64_t *offsets, uint64_t *n_bytes);

// ---- readers (Worker.java:223: DirectoryReader.open on the last commit per
// request; the hits' stored fields are read from that same reader, :234-238)
struct tfidf_reader {
  tfidf_index *ix;
  std::shared_ptr<Snapshot> S;
  std::shared_ptr<StatsView> V;
};

extern "C" int tfidf_reader_open(tfidf_index *ix, tfidf_reader **out) {
  if (!ix || !out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  *out = nullptr;
  std::shared_ptr<StatsView> v;
  std::shared_ptr<Snapshot> S = current(ix, &v);
  if (!S) return fail(TFIDF_E_STATE, "no commit to read");
  *out = new tfidf_reader{ix, std::move(S), std::move(v)};
  return TFIDF_OK;
}

extern "C" int tfidf_reader_close(tfidf_reader *rd) {
  delete rd;
  return TFIDF_OK;
}

extern "C" int tfidf_reader_info(const tfidf_reader *rd, uint64_t *generation, uint64_t *num_docs) {
  if (!rd) return fail(TFIDF_E_INVALID_ARG, "NULL reader");
  if (generation) *generation = rd->S->generation;
  if (num_docs) *num_docs = rd->S->n_docs;
  return TFIDF_OK;
}

extern "C" int tfidf_reader_search(tfidf_reader *rd, const uint8_t *q, uint64_t q_len, uint32_t k, uint32_t *doc_ids,
                                   float *scores, uint64_t cap, uint64_t *n_out) {
  if (!rd || (!q && q_len) || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  *n_out = 0;
  return search_on(rd->ix, *rd->S, *rd->V, q, q_len, k, doc_ids, scores, cap, n_out);
}

extern "C" int tfidf_reader_doc_keys(const tfidf_reader *rd, uint8_t *buf, uint64_t cap, uint64_t *offsets,
                                     uint64_t *n_bytes) {
  if (!rd || !n_bytes || !offsets) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  return doc_keys_of(rd->S.get(), buf, cap, offsets, n_bytes);
}

extern "C" int tfidf_reader_doc_key(const tfidf_reader *rd, uint64_t doc, uint8_t *buf, uint64_t cap,
                                    uint64_t *n_out) {
  if (!rd || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  if (doc >= rd->S->n_docs) return fail(TFIDF_E_INVALID_ARG, "doc out of range");
  std::string k;
  rd->S->keys.key(rd->S->staged_of(doc), &k);
  *n_out = k.size();
  if (k.size() > cap) return fail(TFIDF_E_BUFFER, "key needs %zu bytes", k.size());
  if (buf && !k.empty()) memcpy(buf, k.data(), k.size());
  return TFIDF_OK;
}

extern "C" int tfidf_search_batch(tfidf_index *ix, const uint8_t *q_utf8, const uint64_t *q_offsets, uint32_t n_q,
                                  uint32_t k, uint32_t *doc_ids, float *scores, uint32_t *counts) {
  if (!ix || !q_offsets || !doc_ids || !scores || !counts) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  if (k == 0 || k > 1024) return fail(TFIDF_E_INVALID_ARG, "batch search needs 1 <= k <= 1024");
  std::shared_ptr<StatsView> view;
  const std::shared_ptr<Snapshot> snap = current(ix, &view);
  if (!snap) return fail(TFIDF_E_STATE, "search before commit");
  Snapshot &S = *snap;
  StatsView &V = *view;
  CtxLease lease(ix);
  if (lease.rc) return lease.rc;
  SearchCtx &X = *lease.c;
  const hipStream_t s = lease.stream();
  DeviceGuard g(ix->cfg.device);
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  if (n_q == 0) return TFIDF_OK;
  if (S.n_docs == 0) {
    memset(counts, 0, (size_t)n_q * 4);
    return TFIDF_OK;
  }
  // Pipelined in chunks: chunk c + 1 is prepared on the host (parse, analysis,
  // dictionary lookups, weights) while chunk c scores on the device; each
  // chunk's results are copied (stream-ordered) into its region of one pinned
  // buffer.  Chunks are ceil-sized, so the first one is the largest and the
  // buffers sized by the query count (cand, cand_n, q_out) are reserved by it;
  // q_in (sized by each chunk's terms) grows with an explicit stream sync in
  // run_scoring.  TFIDF_BATCH_CHUNKS overrides.
  // 10 k queries at cfg 2 (tools/gpu_batch_ab.sh): 1 chunk 7.6 ms end to end
  // (prepare 1.5 on the pool, device 5.65), 2 chunks 7.0 (device 6.05), 4
  // chunks 7.45 (device 6.9: every chunk pays the unit kernels' tail)
  // Chunks interleave the queries (chunk c: queries c, c + n_chunks, ...), so
  // each holds the batch's mix of heavy (k_score_units) and light
  // (k_score_wunits) queries and its two concurrent kernels end together
  // (round 6; a contiguous split gave cfg 2's two chunks 3.0 / 1.4 ms and
  // 1.2 / 2.6 ms of heavy / light work: 5.6 ms device)
  uint32_t n_chunks = n_q >= 4096 ? 2 : 1;
  if (const char *e = knob("TFIDF_BATCH_CHUNKS")) n_chunks = (uint32_t)std::max(1, std::min(atoi(e), 64));
  n_chunks = std::max(1u, std::min(n_chunks, n_q));
  const size_t words = (size_t)2 * n_q * k + n_q;
  HIP_TRY(X.q_res.resize(words));
  double t_prep = 0, t_sub = 0;
  bool any = false;
  uint32_t c0 = 0;                                       // results of chunk c start at row c0
  std::vector<uint8_t> cq;                               // chunk c's queries, contiguous
  std::vector<uint64_t> co;
  for (uint32_t c = 0; c < n_chunks; c++) {
    const uint32_t nc = (n_q - c + n_chunks - 1) / n_chunks;   // the first chunk is the largest
    const auto ta = clk::now();
    const uint8_t *cu = q_utf8;
    const uint64_t *coffs = q_offsets;
    if (n_chunks > 1) {
      cq.clear();
      co.assign(1, 0);
      for (uint32_t i = 0; i < nc; i++) {
        const uint32_t q = c + i * n_chunks;
        cq.insert(cq.end(), q_utf8 + q_offsets[q], q_utf8 + q_offsets[q + 1]);
        co.push_back(cq.size());
      }
      cu = cq.data();
      coffs = co.data();
    }
    QueryBatch qb;
    if (int e = prepare_batch(ix, S, V, cu, coffs, nc, &qb)) { X.q_rec_start = true; return e; }
    const auto tb = clk::now();
    uint32_t *hres = X.q_res.data() + (size_t)2 * c0 * k + c0;
    if (qb.slot.empty()) {
      memset(hres + (size_t)2 * nc * k, 0, (size_t)nc * 4);   // no term of the chunk is present
    } else {
      X.q_rec_start = !any;
      const int rc = run_scoring(ix, S, V, X, s, qb, nc, k);
      X.q_rec_start = true;
      if (rc) return rc;
      HIP_TRY(hipMemcpyAsync(hres, X.res_doc, ((size_t)2 * nc * k + nc) * 4, hipMemcpyDeviceToHost, s));
      any = true;
    }
    t_prep += std::chrono::duration<double, std::milli>(tb - ta).count();
    t_sub += std::chrono::duration<double, std::milli>(clk::now() - tb).count();
    c0 += nc;
  }
  const auto t2 = clk::now();
  HIP_TRY(hipStreamSynchronize(s));
  X.q_in_pending = false;
  const auto t3 = clk::now();
  c0 = 0;
  for (uint32_t c = 0; c < n_chunks; c++) {
    const uint32_t nc = (n_q - c + n_chunks - 1) / n_chunks;
    const uint32_t *hres = X.q_res.data() + (size_t)2 * c0 * k + c0;
    for (uint32_t i = 0; i < nc; i++) {
      const uint32_t q = c + i * n_chunks;
      memcpy(doc_ids + (size_t)q * k, hres + (size_t)i * k, (size_t)k * 4);
      memcpy(scores + (size_t)q * k, hres + (size_t)nc * k + (size_t)i * k, (size_t)k * 4);
      counts[q] = hres[(size_t)2 * nc * k + i];
    }
    c0 += nc;
  }
  const float ms_total = any ? qev_ms(X, QEV_0, QEV_2) : 0.0f;
  set_last_ms(ix, any ? qev_ms(X, QEV_0, QEV_1) : 0.0f, ms_total);
  if (knob("TFIDF_HOST_TIMING")) {          // profiling only
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    fprintf(stderr, "batch %u (%u chunks): prepare %.3f  submit %.3f  wait %.3f  copy-out %.3f  total %.3f ms (device %.3f)\n",
            n_q, n_chunks, t_prep, t_sub, ms(t2, t3), ms(t3, clk::now()), ms(t0, clk::now()), ms_total);
  }
  return TFIDF_OK;
}

// Concurrent single searches (the reference's Worker.processDocuments runs on
// concurrent request threads, Worker.java:175-186).  Requests queue up; the
// first caller to find no batch forming leads one: it waits wait_us for
// companions, takes every queued request (up to cq_max), runs them
// through the batched scorer (tfidf_search_batch: one launch for all) and
// hands each caller its own top-k; callers arriving meanwhile form the next
// batch.  Results are those of tfidf_search(k) for each query, including its
// errors (a query that does not parse gets TFIDF_E_QUERY_SYNTAX, not []).
struct CoalesceReq {
  const uint8_t *q;
  uint64_t len;
  uint32_t k;
  uint32_t *docs;
  float *scores;
  uint64_t cap;
  uint64_t *n_out;
  int rc;
  std::string err;
  bool done;
  bool taken;        // in a batch a leader took (waits for that batch, never leads)
};

// One coalesced batch: queries that do not parse answer as tfidf_search
// would; the rest go through one tfidf_search_batch launch.
static void coalesced_run(tfidf_index *ix, const std::vector<CoalesceReq *> &batch) {
  std::vector<CoalesceReq *> run;
  std::vector<uint8_t> text;
  std::vector<uint64_t> offs{0};
  uint32_t kmax = 0;
  for (CoalesceReq *c : batch) {
    QueryPlan plan;
    const int prc = parse_query(c->q, c->len, &plan);
    if (prc == kQBadUtf8 || prc == kQSyntax) {
      c->rc = prc == kQBadUtf8 ? TFIDF_E_UNSUPPORTED_QUERY : TFIDF_E_QUERY_SYNTAX;
      c->err = prc == kQBadUtf8 ? "query is not valid UTF-8"
                                : "query does not parse (QueryParser ParseException / TooManyClauses)";
      *c->n_out = 0;
      continue;
    }
    run.push_back(c);
    text.insert(text.end(), c->q, c->q + c->len);
    offs.push_back(text.size());
    kmax = std::max(kmax, c->k);
  }
  if (run.empty()) return;
  std::vector<uint32_t> docs((size_t)run.size() * kmax), counts(run.size());
  std::vector<float> sc((size_t)run.size() * kmax);
  const int rc = tfidf_search_batch(ix, text.data(), offs.data(), (uint32_t)run.size(), kmax, docs.data(), sc.data(),
                                    counts.data());
  const std::string err = rc != TFIDF_OK ? std::string(tfidf_last_error()) : std::string();
  for (size_t i = 0; i < run.size(); i++) {
    CoalesceReq *c = run[i];
    if (rc != TFIDF_OK) { c->rc = rc; c->err = err; *c->n_out = 0; continue; }
    const uint64_t n = std::min<uint64_t>(counts[i], c->k);     // a prefix of the kmax list = the top-k
    *c->n_out = n;
    if (n > c->cap) { c->rc = TFIDF_E_BUFFER; c->err = "result buffer too small"; continue; }
    memcpy(c->docs, docs.data() + i * kmax, n * 4);
    memcpy(c->scores, sc.data() + i * kmax, n * 4);
  }
}


extern "C" int tfidf_search_coalesced(tfidf_index *ix, const uint8_t *q, uint64_t q_len, uint32_t k, uint32_t *doc_ids,
                                      float *scores, uint64_t cap, uint64_t *n_out, uint32_t wait_us) {
  if (!ix || (!q && q_len) || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  if (k == 0 || k > 1024) return fail(TFIDF_E_INVALID_ARG, "coalesced search needs 1 <= k <= 1024 (all hits: tfidf_search)");
  CoalesceReq r{q, q_len, k, doc_ids, scores, cap, n_out, TFIDF_OK, std::string(), false, false};
  std::unique_lock<std::mutex> lk(ix->cq_mu);
  ix->cq.push_back(&r);
  bool slept = false;
  for (;;) {
    // served by a leader, or not yet taken and no batch is forming: lead one.
    // A request a running leader took waits for that leader (taking part in
    // the next batch would run an empty one).  A leader whose own request did
    // not fit its (capped) batch comes back here; requests left over after a
    // capped batch are woken and one of their callers leads next.
    ix->cq_cv.wait(lk, [&] { return r.done || (!r.taken && !ix->cq_leader); });
    if (r.done) break;
    ix->cq_leader = true;
    if (wait_us && !slept) {
      slept = true;
      lk.unlock();
      std::this_thread::sleep_for(std::chrono::microseconds(wait_us));
      lk.lock();
    }
    const size_t take = std::min(ix->cq.size(), ix->cq_max);   // >= 1: r itself is queued
    std::vector<CoalesceReq *> batch(ix->cq.begin(), ix->cq.begin() + take);
    ix->cq.erase(ix->cq.begin(), ix->cq.begin() + take);
    for (CoalesceReq *c : batch) c->taken = true;
    ix->cq_leader = false;                                // later arrivals lead the next batch
    if (!ix->cq.empty()) ix->cq_cv.notify_all();
    lk.unlock();
    coalesced_run(ix, batch);
    lk.lock();
    ix->cq_batches++;
    ix->cq_queries += batch.size();
    for (CoalesceReq *c : batch) c->done = true;
    ix->cq_cv.notify_all();
  }
  lk.unlock();
  if (r.rc != TFIDF_OK) return fail(r.rc, "%s", r.err.c_str());
  return TFIDF_OK;
}

extern "C" int tfidf_set_query_timing(tfidf_index *ix, int on) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL index");
  ix->q_timing = on != 0;
  return TFIDF_OK;
}

extern "C" int tfidf_last_search_ms(const tfidf_index *ix, float *ms_scoring, float *ms_total) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL index");
  std::lock_guard<std::mutex> lk(const_cast<tfidf_index *>(ix)->ms_mu);
  if (ms_scoring) *ms_scoring = ix->last_ms_scoring;
  if (ms_total) *ms_total = ix->last_ms_total;
  return TFIDF_OK;
}

extern "C" int tfidf_set_stream(tfidf_index *ix, void *stream) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard g(ix->cfg.device);
  HIP_TRY(hipStreamSynchronize(ix->stream));
  ix->stream = stream == TFIDF_OWN_STREAM ? ix->own_stream : static_cast<hipStream_t>(stream);
  ix->user_stream = stream == TFIDF_OWN_STREAM ? nullptr : static_cast<hipStream_t>(stream);
  return TFIDF_OK;
}

static int batch_keys_on(tfidf_index *ix, Snapshot &S, StatsView &V, const uint8_t *q_utf8,
                         const uint64_t *q_offsets, uint32_t n_q, uint32_t k, uint64_t doc_base, void *d_keys) {
  if (!ix || !q_offsets || (n_q && !d_keys)) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  if (k == 0 || k > 1024) return fail(TFIDF_E_INVALID_ARG, "1 <= k <= 1024");
  CtxLease lease(ix);
  if (lease.rc) return lease.rc;
  SearchCtx &X = *lease.c;
  const hipStream_t s = lease.stream();
  DeviceGuard g(ix->cfg.device);
  if (n_q == 0) return TFIDF_OK;
  QueryBatch qb;
  if (int e = prepare_batch(ix, S, V, q_utf8, q_offsets, n_q, &qb)) return e;
  if (S.n_docs == 0 || qb.slot.empty()) {
    HIP_TRY(hipMemsetAsync(d_keys, 0, (size_t)n_q * k * 8, s));
    HIP_TRY(hipStreamSynchronize(s));
    return TFIDF_OK;
  }
  int rc = run_scoring(ix, S, V, X, s, qb, n_q, k);
  if (rc) return rc;
  HIP_TRY(launch_pack_keys(X.res_doc, X.res_score, X.res_n, n_q, k,
                           doc_base, static_cast<uint64_t *>(d_keys), s));
  HIP_TRY(hipStreamSynchronize(s));
  set_last_ms(ix, qev_ms(X, QEV_0, QEV_1), qev_ms(X, QEV_0, QEV_2));
  return TFIDF_OK;
}

extern "C" int tfidf_search_batch_keys_device(tfidf_index *ix, const uint8_t *q_utf8, const uint64_t *q_offsets,
                                              uint32_t n_q, uint32_t k, uint64_t doc_base, void *d_keys) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::shared_ptr<StatsView> view;
  const std::shared_ptr<Snapshot> snap = current(ix, &view);
  if (!snap) return fail(TFIDF_E_STATE, "search before commit");
  return batch_keys_on(ix, *snap, *view, q_utf8, q_offsets, n_q, k, doc_base, d_keys);
}

static int all_keys_on(tfidf_index *ix, Snapshot &S, StatsView &V, const uint8_t *q, uint64_t q_len,
                       uint64_t doc_base, void *d_keys, uint64_t cap, uint64_t *n_out) {
  if (!ix || (!q && q_len) || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  *n_out = 0;
  CtxLease lease(ix);
  if (lease.rc) return lease.rc;
  SearchCtx &X = *lease.c;
  const hipStream_t s = lease.stream();
  if (cap < S.n_docs || (S.n_docs && !d_keys))
    return fail(TFIDF_E_BUFFER, "the key buffer needs num_docs = %llu entries", (unsigned long long)S.n_docs);
  DeviceGuard g(ix->cfg.device);
  PreparedQuery pq;
  int rc = prepare_query(S, V, q, q_len, &pq);
  if (rc) return rc;
  if (pq.slot.empty() || S.n_docs == 0) return TFIDF_OK;
  QueryBatch qb;
  qb.add(pq);
  rc = run_scoring(ix, S, V, X, s, qb, 1, 0);
  if (rc) return rc;
  const uint32_t R = S.n_blocks;
  HIP_TRY(X.hits_c.reserve((size_t)R * kBlockDocs * 8 + 8));
  HIP_TRY(X.hits_s.reserve((size_t)R * kBlockDocs * 8 + 8));
  HIP_TRY(X.hits_P.reserve(((size_t)R + 1) * 8));
  HIP_TRY(launch_hits_order(X.hits.as<uint64_t>(), X.hits_n.as<uint32_t>(), R, X.hits_P.as<uint64_t>(),
                            X.hits_c.as<uint64_t>(), X.hits.as<uint64_t>(), X.hits_s.as<uint64_t>(), nullptr, nullptr,
                            static_cast<uint64_t *>(d_keys), doc_base, hits_bound(S, pq), ix->num_cus * 4, s));
  if (X.q_timing) HIP_TRY(hipEventRecord(X.ev[QEV_2], s));
  HIP_TRY(hipMemcpyAsync(n_out, X.hits_P.as<uint64_t>() + R, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  set_last_ms(ix, qev_ms(X, QEV_0, QEV_1), qev_ms(X, QEV_0, QEV_2));
  return TFIDF_OK;
}

extern "C" int tfidf_search_all_keys_device(tfidf_index *ix, const uint8_t *q, uint64_t q_len, uint64_t doc_base,
                                            void *d_keys, uint64_t cap, uint64_t *n_out) {
  if (!ix || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  *n_out = 0;
  std::shared_ptr<StatsView> view;
  const std::shared_ptr<Snapshot> snap = current(ix, &view);
  if (!snap) return fail(TFIDF_E_STATE, "search before commit");
  return all_keys_on(ix, *snap, *view, q, q_len, doc_base, d_keys, cap, n_out);
}

// the same on a reader's pinned snapshot (the node-level searches: status
// check, local search and document count from one snapshot)
int tfidf::reader_batch_keys_device(tfidf_reader *rd, const uint8_t *q_utf8, const uint64_t *q_offsets, uint32_t n_q,
                                    uint32_t k, uint64_t doc_base, void *d_keys) {
  return batch_keys_on(rd->ix, *rd->S, *rd->V, q_utf8, q_offsets, n_q, k, doc_base, d_keys);
}
int tfidf::reader_all_keys_device(tfidf_reader *rd, const uint8_t *q, uint64_t q_len, uint64_t doc_base, void *d_keys,
                                  uint64_t cap, uint64_t *n_out) {
  return all_keys_on(rd->ix, *rd->S, *rd->V, q, q_len, doc_base, d_keys, cap, n_out);
}

// ---------------------------------------------------------------------------
// inspection

extern "C" int tfidf_doc_key(const tfidf_index *ix, uint64_t doc, uint8_t *buf, uint64_t cap, uint64_t *n_out) {
  if (!ix || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  const std::shared_ptr<Snapshot> S = current(ix);
  if (!S || doc >= S->n_docs) return fail(TFIDF_E_INVALID_ARG, "doc out of range");
  std::string k;
  S->keys.key(S->staged_of(doc), &k);
  *n_out = k.size();
  if (k.size() > cap) return fail(TFIDF_E_BUFFER, "key needs %zu bytes", k.size());
  if (buf && !k.empty()) memcpy(buf, k.data(), k.size());
  return TFIDF_OK;
}

static int doc_keys_of(const Snapshot *S, uint8_t *buf, uint64_t cap, uint64_t *offsets, uint64_t *n_bytes) {
  uint64_t need = 0;
  for (uint64_t d = 0; d < S->n_docs; d++) need += S->keys.key_len(S->staged_of(d));
  *n_bytes = need;
  if (need > cap || (need && !buf)) return fail(TFIDF_E_BUFFER, "keys need %llu bytes", (unsigned long long)need);
  uint64_t p = 0;
  offsets[0] = 0;
  std::string k;
  for (uint64_t d = 0; d < S->n_docs; d++) {
    S->keys.key(S->staged_of(d), &k);
    memcpy(buf + p, k.data(), k.size());
    p += k.size();
    offsets[d + 1] = p;
  }
  return TFIDF_OK;
}

extern "C" int tfidf_doc_keys(const tfidf_index *ix, uint8_t *buf, uint64_t cap, uint64_t *offsets,
                              uint64_t *n_bytes) {
  if (!ix || !n_bytes || !offsets) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  const std::shared_ptr<Snapshot> S = current(ix);
  if (!S) return fail(TFIDF_E_STATE, "not committed");
  return doc_keys_of(S.get(), buf, cap, offsets, n_bytes);
}

extern "C" int tfidf_malformed_docs(const tfidf_index *ix, uint64_t *docs, uint64_t cap, uint64_t *n_out) {
  if (!ix || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  const std::shared_ptr<Snapshot> S = current(ix);
  if (!S) return fail(TFIDF_E_STATE, "not committed");
  *n_out = S->malformed.size();
  if (S->malformed.size() > cap || (cap && !docs && !S->malformed.empty()))
    return fail(TFIDF_E_BUFFER, "need %zu entries", S->malformed.size());
  for (size_t i = 0; i < S->malformed.size(); i++) docs[i] = S->malformed[i];
  return TFIDF_OK;
}

extern "C" int tfidf_doc_len(tfidf_index *ix, uint64_t doc, uint32_t *len, uint8_t *norm) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL index");
  const std::shared_ptr<Snapshot> S = current(ix);
  if (!S || doc >= S->n_docs) return fail(TFIDF_E_INVALID_ARG, "doc out of range");
  DeviceGuard g(ix->cfg.device);
  uint32_t l = 0;
  uint8_t n = 0;
  HIP_TRY(hipMemcpy(&l, S->doc_len.as<uint32_t>() + doc, 4, hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(&n, S->doc_norm.as<uint8_t>() + doc, 1, hipMemcpyDeviceToHost));
  if (len) *len = l;
  if (norm) *norm = n;
  return TFIDF_OK;
}

extern "C" int tfidf_doc_terms(tfidf_index *ix, uint64_t doc, char *terms, uint64_t terms_cap, uint32_t *tfs,
                               uint64_t cap, uint64_t *n_out) {
  if (!ix || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap || doc >= snap->n_docs) return fail(TFIDF_E_INVALID_ARG, "doc out of range");
  Snapshot &S = *snap;
  DeviceGuard g(ix->cfg.device);
  uint32_t nu = 0;
  HIP_TRY(hipMemcpy(&nu, S.doc_nuniq.as<uint32_t>() + doc, 4, hipMemcpyDeviceToHost));
  const uint64_t st = S.staged_of(doc);
  uint64_t off_st = 0;                               // the document's corpus offset (its CSR row base)
  HIP_TRY(hipMemcpy(&off_st, S.offsets->as<uint64_t>() + st, 8, hipMemcpyDeviceToHost));
  const uint64_t base = (off_st + st) >> 1;          // csr_row_base
  // packed entries: the row's range segments (rsplit) give each slot's range
  std::vector<uint32_t> ent(nu), col(nu), tf(nu), split(S.R);
  if (nu) {
    HIP_TRY(hipMemcpy(ent.data(), S.csr.as<uint32_t>() + base, nu * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(split.data(), S.rsplit.as<uint32_t>() + doc * S.R, S.R * 4, hipMemcpyDeviceToHost));
  }
  const uint32_t rs = S.range_shift, esc = csr_esc_value(rs);
  for (uint32_t i = 0, r = 0; i < nu; i++) {
    while (r + 1 < S.R && i >= split[r]) r++;
    col[i] = (r << rs) | csr_local(ent[i], rs);
    const uint32_t f = csr_tf_field(ent[i], rs);
    tf[i] = f == esc ? csr_esc_tf(S.h_esc.data(), S.h_esc.size(), base + i) : f;
  }
  std::vector<std::pair<std::string, uint32_t>> rows;
  for (uint32_t i = 0; i < nu; i++) {
    std::string t;
    if (int rc = slot_term(S, col[i], &t)) return rc;
    rows.emplace_back(std::move(t), tf[i]);
  }
  std::sort(rows.begin(), rows.end());
  uint64_t need = 0;
  for (auto &r : rows) need += r.first.size() + 1;
  *n_out = rows.size();
  if (need > terms_cap || rows.size() > cap) return fail(TFIDF_E_BUFFER, "buffers too small");
  uint64_t p = 0;
  for (size_t i = 0; i < rows.size(); i++) {
    memcpy(terms + p, rows[i].first.c_str(), rows[i].first.size() + 1);
    p += rows[i].first.size() + 1;
    tfs[i] = rows[i].second;
  }
  return TFIDF_OK;
}

extern "C" int tfidf_term_df(tfidf_index *ix, const uint8_t *term, uint64_t len, uint64_t *df_local,
                             uint64_t *df_effective) {
  if (!ix || (!term && len)) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::shared_ptr<StatsView> V;
  const std::shared_ptr<Snapshot> S = current(ix, &V);
  if (!S) return fail(TFIDF_E_STATE, "not committed");
  if (int e = V->wait_gdf()) return e;
  DeviceGuard g(ix->cfg.device);
  std::string t((const char *)term, len);
  const uint32_t s = lookup_term(*S, t);
  const uint64_t l = s == kInvalidSlot ? 0 : S->h_df[s];
  if (df_local) *df_local = l;
  if (df_effective) *df_effective = (s != kInvalidSlot && V->global) ? V->gdf[s] : l;
  return TFIDF_OK;
}

extern "C" int tfidf_term_key(const uint8_t *term, uint64_t len, uint64_t *lo, uint64_t *hi) {
  if ((!term && len) || !lo || !hi) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::string t((const char *)term, len);
  term_key(t, lo, hi);
  return TFIDF_OK;
}

extern "C" int tfidf_analyze(const uint8_t *text, uint64_t len, char *out, uint64_t cap, uint64_t *n_tokens,
                             uint64_t *n_bytes) {
  if ((!text && len) || !n_tokens || !n_bytes || (!out && cap)) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::vector<std::string> toks;
  if (!analyze(text, len, &toks)) return fail(TFIDF_E_UNSUPPORTED_INPUT, "text is not valid UTF-8");
  uint64_t need = 0;
  for (auto &t : toks) need += t.size() + 1;
  *n_tokens = toks.size();
  *n_bytes = need;
  if (need > cap) return fail(TFIDF_E_BUFFER, "buffer too small");
  uint64_t p = 0;
  for (auto &t : toks) {
    memcpy(out + p, t.data(), t.size());
    out[p + t.size()] = 0;
    p += t.size() + 1;
  }
  return TFIDF_OK;
}

// ---------------------------------------------------------------------------
// GLOBAL statistics

extern "C" int tfidf_vocab_size(const tfidf_index *ix, uint64_t *n) {
  if (!ix || !n) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  const std::shared_ptr<Snapshot> S = current(ix);
  *n = S ? S->num_terms : 0;
  return TFIDF_OK;
}

extern "C" int tfidf_vocab_export_device(tfidf_index *ix, void *d_keys, void *d_df, uint64_t cap, uint64_t *n_out) {
  if (!ix || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap) return fail(TFIDF_E_STATE, "not committed");
  const Snapshot &S = *snap;
  DeviceGuard g(ix->cfg.device);
  *n_out = S.num_terms;
  if (S.num_terms > cap) return fail(TFIDF_E_BUFFER, "need %llu keys", (unsigned long long)S.num_terms);
  // sorted (hi, lo) key list of this shard + df, assembled from the host mirror
  std::vector<std::pair<std::pair<uint64_t, uint64_t>, uint32_t>> v;
  v.reserve(S.num_terms);
  for (uint32_t s = 0; s < S.C; s++)
    if (S.h_dict[s])
      v.push_back({{S.h_dict[(size_t)S.C + s], S.h_dict[s]}, S.h_df[s]});
  std::sort(v.begin(), v.end());
  std::vector<uint64_t> keys(2 * v.size());
  std::vector<uint32_t> df(v.size());
  for (size_t i = 0; i < v.size(); i++) {
    keys[2 * i] = v[i].first.second;
    keys[2 * i + 1] = v[i].first.first;
    df[i] = v[i].second;
  }
  if (!v.empty()) {
    if (d_keys) HIP_TRY(hipMemcpy(d_keys, keys.data(), keys.size() * 8, hipMemcpyHostToDevice));
    if (d_df) HIP_TRY(hipMemcpy(d_df, df.data(), df.size() * 4, hipMemcpyHostToDevice));
  }
  return TFIDF_OK;
}

extern "C" int tfidf_vocab_export(tfidf_index *ix, uint64_t *keys, uint32_t *df_local, uint32_t *df_effective,
                                  uint64_t cap, uint64_t *n_out) {
  if (!ix || !n_out) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::shared_ptr<StatsView> view;
  const std::shared_ptr<Snapshot> snap = current(ix, &view);
  if (!snap) return fail(TFIDF_E_STATE, "not committed");
  const Snapshot &S = *snap;
  StatsView &V = *view;
  if (int e = V.wait_gdf()) return e;
  *n_out = S.num_terms;
  if (S.num_terms > cap) return fail(TFIDF_E_BUFFER, "need %llu terms", (unsigned long long)S.num_terms);
  std::vector<std::pair<std::pair<uint64_t, uint64_t>, uint32_t>> v;   // ((hi, lo), slot)
  v.reserve(S.num_terms);
  for (uint32_t s = 0; s < S.C; s++)
    if (S.h_dict[s]) v.push_back({{S.h_dict[(size_t)S.C + s], S.h_dict[s]}, s});
  std::sort(v.begin(), v.end());
  for (size_t i = 0; i < v.size(); i++) {
    const uint32_t s = v[i].second;
    if (keys) { keys[2 * i] = v[i].first.second; keys[2 * i + 1] = v[i].first.first; }
    if (df_local) df_local[i] = S.h_df[s];
    if (df_effective) df_effective[i] = V.global ? V.gdf[s] : S.h_df[s];
  }
  return TFIDF_OK;
}

extern "C" int tfidf_vocab_canonicalize_device(tfidf_index *ix, const void *d_all_keys, uint64_t n_all,
                                               void *d_df_canonical, uint64_t cap, uint64_t *n_canonical) {
  if (!ix || !n_canonical) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap) return fail(TFIDF_E_STATE, "not committed");
  const Snapshot &S = *snap;
  DeviceGuard g(ix->cfg.device);
  hipStream_t s = ix->stream;
  DevBuf canon;
  HIP_TRY(canon.reserve(n_all * 16 + 16));
  uint64_t nu = 0;
  HIP_TRY(sort_unique_keys128((const uint64_t *)d_all_keys, n_all, canon.as<uint64_t>(), &nu, s));
  *n_canonical = nu;
  if (nu > cap) { canon.release(); return fail(TFIDF_E_BUFFER, "need %llu canonical slots", (unsigned long long)nu); }
  HIP_TRY(ix->canon_of_slot.reserve((size_t)S.C * 4));
  HIP_TRY(slot_to_canon(S.dict.as<uint64_t>(), S.C, canon.as<uint64_t>(), nu, ix->canon_of_slot.as<uint32_t>(), s));
  if (d_df_canonical) {
    HIP_TRY(hipMemsetAsync(d_df_canonical, 0, nu * 4, s));
    HIP_TRY(scatter_df_canon(S.df_dev(), ix->canon_of_slot.as<uint32_t>(), S.C, (uint32_t *)d_df_canonical, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  canon.release();
  ix->n_canon = nu;
  return TFIDF_OK;
}

// The device-buffer exchange calls run on ix->stream.  On a caller's stream
// (tfidf_set_stream) they stay asynchronous: the caller's allocator orders
// its buffers on that stream.  On the index's own stream nothing orders the
// caller's buffers against the work, so the call returns only once the work
// that reads or writes them is done.
static int exchange_done(tfidf_index *ix) {
  if (ix->stream == ix->own_stream && hipStreamSynchronize(ix->stream) != hipSuccess)
    return fail(TFIDF_E_HIP, "hipStreamSynchronize failed");
  return TFIDF_OK;
}

static int vocab_partition(tfidf_index *ix, uint32_t n_ranks, void *d_records, uint64_t cap, void *d_counts,
                           uint64_t *n_out, bool sync) {
  if (!ix || !n_out || !d_counts || n_ranks == 0 || n_ranks > 1024)
    return fail(TFIDF_E_INVALID_ARG, "NULL argument or n_ranks not in [1, 1024]");
  std::lock_guard<std::mutex> lk(ix->mu);
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap) return fail(TFIDF_E_STATE, "not committed");
  const Snapshot &S = *snap;
  DeviceGuard g(ix->cfg.device);
  *n_out = S.num_terms;
  if (S.num_terms > cap) return fail(TFIDF_E_BUFFER, "need %llu records", (unsigned long long)S.num_terms);
  if (S.num_terms && !d_records) return fail(TFIDF_E_INVALID_ARG, "NULL records");
  hipStream_t s = ix->stream;
  HIP_TRY(ix->vcounts.reserve((size_t)n_ranks * 8 + 64));
  HIP_TRY(ix->sent_slot.reserve(S.num_terms * 4 + 4));
  uint32_t *cnt = ix->vcounts.as<uint32_t>(), *cur = cnt + n_ranks;
  HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)n_ranks * 4, s));
  HIP_TRY(vocab_count(S.dict.as<uint64_t>(), S.C, n_ranks, cnt, s));
  HIP_TRY(vocab_starts(cnt, n_ranks, cur, static_cast<uint64_t *>(d_counts), s));
  HIP_TRY(vocab_scatter(S.dict.as<uint64_t>(), S.df_dev(), S.C, n_ranks, cur, (uint64_t *)d_records,
                        ix->sent_slot.as<uint32_t>(), s));
  ix->n_sent = S.num_terms;
  return sync ? exchange_done(ix) : TFIDF_OK;          // asynchronous on a caller's stream
}
extern "C" int tfidf_vocab_partition_device(tfidf_index *ix, uint32_t n_ranks, void *d_records, uint64_t cap,
                                            void *d_counts, uint64_t *n_out) {
  return vocab_partition(ix, n_ranks, d_records, cap, d_counts, n_out, true);
}
int tfidf::vocab_partition_async(tfidf_index *ix, uint32_t n_ranks, void *d_records, uint64_t cap, void *d_counts,
                                 uint64_t *n_out) {
  return vocab_partition(ix, n_ranks, d_records, cap, d_counts, n_out, false);
}

static int vocab_reduce_dev(tfidf_index *ix, const void *d_records, uint64_t n, void *d_df_out, void *d_n_unique,
                            bool sync) {
  if (!ix || (n && (!d_records || !d_df_out))) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  DeviceGuard g(ix->cfg.device);
  hipStream_t s = ix->stream;
  if (n >= (1ull << 30)) return fail(TFIDF_E_CAPACITY, "too many vocabulary records");
  if (n == 0) {
    if (d_n_unique) HIP_TRY(hipMemsetAsync(d_n_unique, 0, 8, s));
    return TFIDF_OK;
  }
  uint64_t T = 1024;
  while (T < 2 * n) T <<= 1;
  HIP_TRY(ix->vt_table.reserve(T * 16));
  HIP_TRY(ix->vt_sum.reserve(T * 4));
  HIP_TRY(ix->vt_rslot.reserve(n * 4));
  HIP_TRY(hipMemsetAsync(ix->vt_table.p, 0, T * 16, s));
  HIP_TRY(hipMemsetAsync(ix->vt_sum.p, 0, T * 4, s));
  HIP_TRY(ix->vnu.reserve(64));
  unsigned long long *nu = reinterpret_cast<unsigned long long *>(d_n_unique ? d_n_unique : ix->vnu.p);   // counted in place
  HIP_TRY(hipMemsetAsync(nu, 0, 8, s));
  HIP_TRY(vocab_reduce((const uint64_t *)d_records, n, ix->vt_table.as<uint64_t>(), (uint32_t)(T - 1),
                       ix->vt_sum.as<uint32_t>(), ix->vt_rslot.as<uint32_t>(), (uint32_t *)d_df_out, nu, s));
  return sync ? exchange_done(ix) : TFIDF_OK;          // asynchronous on a caller's stream
}
extern "C" int tfidf_vocab_reduce_device(tfidf_index *ix, const void *d_records, uint64_t n, void *d_df_out,
                                         void *d_n_unique) {
  return vocab_reduce_dev(ix, d_records, n, d_df_out, d_n_unique, true);
}
int tfidf::vocab_reduce_async(tfidf_index *ix, const void *d_records, uint64_t n, void *d_df_out, void *d_n_unique) {
  return vocab_reduce_dev(ix, d_records, n, d_df_out, d_n_unique, false);
}

// A new statistics view for the current snapshot (the GLOBAL setters): built
// aside, complete on the device (norm cache uploaded) before searches see it.
// The view it replaces is kept as the next setter's spare.  async: the cache
// upload (and whatever the caller queued for the view before) completes
// behind the view's event, which every search waits for before its first use
// (StatsView::wait_gdf) — the setter itself never waits for the device.
static int publish_view(tfidf_index *ix, Snapshot &S, const std::shared_ptr<StatsView> &v, bool async = false) {
  if (int e = upload_cache(ix->cfg, *v, ix->stream, !async)) return e;
  if (async) {
    std::lock_guard<std::mutex> gl(v->gdf_mu);
    HIP_TRY(hipEventRecord(v->gdf_ev, ix->stream));
    v->gdf_pending = true;
  }
  std::shared_ptr<StatsView> old;
  {
    std::lock_guard<std::mutex> sl(ix->snap_mu);
    old = std::move(S.stats);
    S.stats = v;
  }
  if (old && old != v) ix->view_spare = std::move(old);
  return TFIDF_OK;
}

// A statistics view to fill: the spare one once no search holds it (ADVICE
// r05: a fresh view per GLOBAL exchange pinned C x 4 bytes of host memory and
// freed the previous view's, which synchronises the device), else a new one.
static std::shared_ptr<StatsView> take_view(tfidf_index *ix) {
  std::shared_ptr<StatsView> v;
  if (ix->view_spare && ix->view_spare.use_count() == 1) {
    v = std::move(ix->view_spare);
    if (v->wait_gdf() != TFIDF_OK) v.reset();          // its last uploads have left h_cache / gdf
  }
  ix->view_spare.reset();
  if (!v) v = std::make_shared<StatsView>(ix->cfg.device);
  v->global = false;
  v->gdf.clear();
  return v;
}

// tfidf_set_global_df_device (sync: the public call, which returns when the
// caller's df buffer has been read on the index's own stream) and its
// asynchronous form for tfidf_dist_global_commit (every buffer is the
// communicator's, ordered on the index's stream).  *generation: the commit
// generation of the snapshot the GLOBAL view was published on.
static int set_global_df(tfidf_index *ix, const void *d_df, uint64_t n, uint64_t doc_count, uint64_t sum_ttf,
                         bool sync, uint64_t *generation) {
  if (!ix || (n && !d_df)) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap) return fail(TFIDF_E_STATE, "not committed");
  Snapshot &S = *snap;
  if (n != ix->n_sent) return fail(TFIDF_E_STATE, "expected %llu records (tfidf_vocab_partition_device)",
                                   (unsigned long long)ix->n_sent);
  DeviceGuard g(ix->cfg.device);
  hipStream_t s = ix->stream;
  std::shared_ptr<StatsView> v = take_view(ix);
  HIP_TRY(ix->gdf_dev.reserve((size_t)S.C * 4));
  HIP_TRY(hipMemsetAsync(ix->gdf_dev.p, 0, (size_t)S.C * 4, s));
  HIP_TRY(vocab_import(ix->sent_slot.as<uint32_t>(), (const uint32_t *)d_df, n, ix->gdf_dev.as<uint32_t>(), s));
  // host mirror for query analysis: copied asynchronously, waited for by the
  // first query (prepare_query) — the exchange itself needs no host sync
  HIP_TRY(v->gdf.resize(S.C));
  HIP_TRY(hipMemcpyAsync(v->gdf.data(), ix->gdf_dev.p, (size_t)S.C * 4, hipMemcpyDeviceToHost, s));
  {
    std::lock_guard<std::mutex> gl(v->gdf_mu);
    HIP_TRY(hipEventRecord(v->gdf_ev, s));
    v->gdf_pending = true;
  }
  v->global = true;
  v->doc_count = doc_count;
  v->sum_ttf = sum_ttf;
  if (generation) *generation = S.generation;
  if (sync) {
    if (int e = exchange_done(ix)) return e;
    return publish_view(ix, S, v);
  }
  return publish_view(ix, S, v, true);
}

extern "C" int tfidf_set_global_df_device(tfidf_index *ix, const void *d_df, uint64_t n, uint64_t doc_count,
                                          uint64_t sum_ttf) {
  return set_global_df(ix, d_df, n, doc_count, sum_ttf, true, nullptr);
}

int tfidf::set_global_df_async(tfidf_index *ix, const void *d_df, uint64_t n, uint64_t doc_count, uint64_t sum_ttf,
                               uint64_t *generation) {
  return set_global_df(ix, d_df, n, doc_count, sum_ttf, false, generation);
}

extern "C" int tfidf_set_global_stats_device(tfidf_index *ix, const void *d_df_canonical, uint64_t n_canonical,
                                             uint64_t doc_count, uint64_t sum_ttf) {
  if (!ix || !d_df_canonical) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap) return fail(TFIDF_E_STATE, "not committed");
  Snapshot &S = *snap;
  if (n_canonical != ix->n_canon) return fail(TFIDF_E_STATE, "canonical vocabulary size mismatch");
  DeviceGuard g(ix->cfg.device);
  hipStream_t s = ix->stream;
  std::shared_ptr<StatsView> v = take_view(ix);
  DevBuf gd;
  HIP_TRY(gd.reserve((size_t)S.C * 4));
  HIP_TRY(gather_df_canon((const uint32_t *)d_df_canonical, ix->canon_of_slot.as<uint32_t>(), S.C,
                          gd.as<uint32_t>(), s));
  HIP_TRY(v->gdf.resize(S.C));
  HIP_TRY(hipMemcpyAsync(v->gdf.data(), gd.p, (size_t)S.C * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  gd.release();
  v->global = true;
  v->doc_count = doc_count;
  v->sum_ttf = sum_ttf;
  return publish_view(ix, S, v);
}

extern "C" int tfidf_set_global_stats(tfidf_index *ix, const uint64_t *keys_lohi, const uint64_t *df, uint64_t n,
                                      uint64_t doc_count, uint64_t sum_ttf) {
  if (!ix || (n && (!keys_lohi || !df))) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(ix->mu);
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap) return fail(TFIDF_E_STATE, "not committed");
  Snapshot &S = *snap;
  DeviceGuard g(ix->cfg.device);
  std::shared_ptr<StatsView> v = take_view(ix);
  HIP_TRY(v->gdf.assign(S.C, 0));
  for (uint32_t s = 0; s < S.C; s++) v->gdf[s] = S.h_df[s];  // keys not listed keep local df
  for (uint64_t i = 0; i < n; i++) {
    const uint32_t s = host_lookup(S, keys_lohi[2 * i], keys_lohi[2 * i + 1]);
    if (s != kInvalidSlot) v->gdf[s] = (uint32_t)df[i];
  }
  v->global = true;
  v->doc_count = doc_count;
  v->sum_ttf = sum_ttf;
  return publish_view(ix, S, v);
}

extern "C" int tfidf_clear_global_stats(tfidf_index *ix) {
  if (!ix) return fail(TFIDF_E_INVALID_ARG, "NULL index");
  std::lock_guard<std::mutex> lk(ix->mu);
  const std::shared_ptr<Snapshot> snap = current(ix);
  if (!snap) return TFIDF_OK;
  Snapshot &S = *snap;
  DeviceGuard g(ix->cfg.device);
  std::shared_ptr<StatsView> v = take_view(ix);
  v->doc_count = S.doc_count;
  v->sum_ttf = S.sum_ttf;
  return publish_view(ix, S, v);
}

// ---------------------------------------------------------------------------
// Leader.start merge (host: it merges per-worker result lists by name)

// String.compareTo order of two UTF-8 names: Java compares UTF-16 code units,
// so a supplementary code point (a surrogate pair, lead 0xD800..0xDBFF)
// sorts below U+E000..U+FFFF although its code point is larger.  Both names
// are walked as UTF-16 code units (a supplementary code point yields its lead,
// then its trail surrogate); a malformed UTF-8 sequence compares by its bytes.
static bool utf8_next(const uint8_t *s, uint64_t n, uint64_t *i, uint32_t *cp) {
  const uint8_t c = s[*i];
  uint32_t len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
  if (!len || *i + len > n) return false;
  uint32_t v = len == 1 ? c : c & (0x7Fu >> len);
  for (uint32_t k = 1; k < len; k++) {
    if ((s[*i + k] & 0xC0) != 0x80) return false;
    v = (v << 6) | (s[*i + k] & 0x3F);
  }
  *i += len;
  *cp = v;
  return true;
}

struct Utf16Units {                // UTF-8 bytes -> UTF-16 code units
  const uint8_t *s;
  uint64_t n, i = 0;
  uint32_t trail = 0;              // pending trail surrogate of a supplementary code point
  bool more() const { return trail || i < n; }
  // next code unit; false (at byte i) if the UTF-8 there is malformed
  bool next(uint32_t *u) {
    if (trail) { *u = trail; trail = 0; return true; }
    uint32_t cp;
    if (!utf8_next(s, n, &i, &cp)) return false;
    if (cp >= 0x10000) {
      *u = 0xD800 + ((cp - 0x10000) >> 10);
      trail = 0xDC00 + ((cp - 0x10000) & 0x3FF);
    } else {
      *u = cp;
    }
    return true;
  }
};

int tfidf::utf16_compare(const uint8_t *a, uint64_t na, const uint8_t *b, uint64_t nb) {
  Utf16Units x{a, na}, y{b, nb};
  while (x.more() && y.more()) {
    const uint64_t i0 = x.i, j0 = y.i;
    uint32_t u, v;
    if (!x.next(&u) || !y.next(&v)) {                     // malformed: bytes from here on
      const uint64_t ra = na - i0, rb = nb - j0;
      const int c = memcmp(a + i0, b + j0, std::min(ra, rb));
      return c ? c : (ra < rb ? -1 : ra > rb);
    }
    if (u != v) return u < v ? -1 : 1;
  }
  return x.more() ? 1 : (y.more() ? -1 : 0);
}

extern "C" int tfidf_sort_names(const uint8_t *names, const uint64_t *offsets, uint64_t n, uint64_t *perm) {
  if (n && (!names || !offsets || !perm)) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  for (uint64_t i = 0; i < n; i++) perm[i] = i;
  std::stable_sort(perm, perm + n, [&](uint64_t x, uint64_t y) {
    return utf16_compare(names + offsets[x], offsets[x + 1] - offsets[x], names + offsets[y],
                         offsets[y + 1] - offsets[y]) < 0;
  });
  return TFIDF_OK;
}

extern "C" int tfidf_leader_merge(const uint8_t *names, const uint64_t *offsets, uint64_t n, const double *scores,
                                  uint64_t *out_first, double *out_sum, uint64_t *n_out) {
  if (!n_out || (n && (!names || !offsets || !scores || !out_first || !out_sum)))
    return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  std::unordered_map<std::string, size_t> pos;
  std::vector<uint64_t> first;
  std::vector<double> sum;
  for (uint64_t i = 0; i < n; i++) {
    std::string k((const char *)names + offsets[i], offsets[i + 1] - offsets[i]);
    auto it = pos.find(k);
    if (it == pos.end()) {                   // HashMap.merge: first value stored as-is
      pos.emplace(std::move(k), sum.size());
      first.push_back(i);
      sum.push_back(scores[i]);
    } else {
      sum[it->second] += scores[i];          // Double::sum in response order
    }
  }
  std::vector<size_t> idx(first.size());
  for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {   // TreeMap<String, Double>: String.compareTo
    const uint64_t x = first[a], y = first[b];
    return utf16_compare(names + offsets[x], offsets[x + 1] - offsets[x], names + offsets[y],
                         offsets[y + 1] - offsets[y]) < 0;
  });
  for (size_t r = 0; r < idx.size(); r++) {
    out_first[r] = first[idx[r]];
    out_sum[r] = sum[idx[r]];
  }
  *n_out = idx.size();
  return TFIDF_OK;
}

// ---------------------------------------------------------------------------
// synthetic corpus

extern "C" int tfidf_synth_corpus(int device, uint64_t seed, uint64_t n_docs, uint64_t doc_base, const double *cdf,
                                  uint32_t V, uint32_t len_min, uint32_t len_max, void **d_text, void **d_offsets,
                                  uint64_t *total_bytes) {
  if (!cdf || !d_text || !d_offsets || !total_bytes || V == 0 || len_max < len_min)
    return fail(TFIDF_E_INVALID_ARG, "bad argument");
  if (len_max >= (1u << 20) - 1) return fail(TFIDF_E_INVALID_ARG, "len_max must be < 2^20 - 1");
  DeviceGuard g(device);
  hipStream_t s;
  HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint32_t G = 1u << 16;
  std::vector<uint32_t> guide(G + 1);
  for (uint32_t i = 0; i <= G; i++) {
    const double u = (double)i / (double)G;
    guide[i] = (uint32_t)(std::upper_bound(cdf, cdf + V, u) - cdf);
    if (guide[i] > V - 1) guide[i] = V - 1;
  }
  DevBuf dcdf, dguide, bytes;
  HIP_TRY(dcdf.reserve((size_t)V * 8));
  HIP_TRY(dguide.reserve((size_t)(G + 1) * 4));
  HIP_TRY(bytes.reserve(n_docs * 8 + 8));
  void *off = nullptr;
  HIP_TRY(hipMalloc(&off, (n_docs + 1) * 8));
  HIP_TRY(hipMemcpyAsync(dcdf.p, cdf, (size_t)V * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(dguide.p, guide.data(), (size_t)(G + 1) * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(synth_doc_lengths(seed, n_docs, doc_base, dcdf.as<double>(), dguide.as<uint32_t>(), V, len_min, len_max,
                            bytes.as<uint64_t>(), s));
  HIP_TRY(exclusive_scan_u64(bytes.as<uint64_t>(), (uint64_t *)off, n_docs, s));
  uint64_t tot = 0;
  HIP_TRY(hipMemcpyAsync(&tot, (uint64_t *)off + n_docs, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  void *txt = nullptr;
  HIP_TRY(hipMalloc(&txt, tot + 128));
  HIP_TRY(hipMemsetAsync(txt, 0, tot + 128, s));
  HIP_TRY(synth_doc_text(seed, n_docs, doc_base, dcdf.as<double>(), dguide.as<uint32_t>(), V, len_min, len_max,
                         (const uint64_t *)off, (uint8_t *)txt, s));
  HIP_TRY(hipStreamSynchronize(s));
  dcdf.release();
  dguide.release();
  bytes.release();
  hipStreamDestroy(s);
  *d_text = txt;
  *d_offsets = off;
  *total_bytes = tot;
  return TFIDF_OK;
}

extern "C" int tfidf_device_free(int device, void *d_ptr) {
  DeviceGuard g(device);
  if (d_ptr) HIP_TRY(hipFree(d_ptr));
  return TFIDF_OK;
}

extern "C" int tfidf_device_copy(int device, void *dst, const void *src, uint64_t bytes, int kind) {
  if ((!dst || !src) && bytes) return fail(TFIDF_E_INVALID_ARG, "NULL argument");
  if (kind != 1 && kind != 2) return fail(TFIDF_E_INVALID_ARG, "kind must be 1 (H2D) or 2 (D2H)");
  DeviceGuard g(device);
  if (bytes) HIP_TRY(hipMemcpy(dst, src, bytes, kind == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost));
  return TFIDF_OK;
}

// ---------------------------------------------------------------------------
// internal accessors for the node-level orchestration (tfidf_dist.hip)

hipStream_t tfidf::index_stream(tfidf_index *ix) { return ix->stream; }
int tfidf::index_device(const tfidf_index *ix) { return ix->cfg.device; }
bool tfidf::index_committed(const tfidf_index *ix) { return current(ix) != nullptr; }
uint64_t tfidf::index_num_docs(const tfidf_index *ix) {
  const std::shared_ptr<Snapshot> S = current(ix);
  return S ? S->n_docs : 0;
}
uint64_t tfidf::index_generation(const tfidf_index *ix) {
  const std::shared_ptr<Snapshot> S = current(ix);
  return S ? S->generation : 0;
}
int tfidf::set_error(int code, const char *msg) { return fail(code, "%s", msg); }
