// tfidf_dist.hip — node level: documents sharded over GPUs, one shard
// (tfidf_index) per GPU, collectives between the shards (include/tfidf.h,
// "Node level").  Replaces the reference's Leader.start fan-out + merge
// (Leader.java:39-92: POST /worker/process to every worker, :51-70; sum per
// name, :73-77; TreeMap order, :80-88) over Worker.searchIndex
// (Worker.java:222-241), with the workers as GPU shards and RCCL collectives
// over xGMI in place of HTTP.
//
//   transports : caller callbacks (host or device buffers), the built-in RCCL
//                communicator (librccl of the HIP runtime this library runs on,
//                loaded at first use), or an in-process host transport for
//                shards of one process that share a device (tests).
//   tfidf_dist_*: per-rank (SPMD) orchestration: GLOBAL statistics by term
//                ownership, top-k / all-hits / batch merges of device merge
//                keys, SHARD mode's name table and Leader-style merge.
//   tfidf_node_*: one process owning every GPU of a device list: a worker
//                thread per shard runs the same per-rank orchestration.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/tfidf.h"
#include "analysis.h"
#include "tfidf_common.h"
#include "tfidf_internal.h"

using namespace tfidf;

namespace {

int errf(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int errf(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return set_error(code, buf);
}

#define DHIP(expr)                                                                                  \
  do {                                                                                              \
    hipError_t _e = (expr);                                                                         \
    if (_e != hipSuccess)                                                                           \
      return errf(TFIDF_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
  } while (0)

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    hipGetDevice(&prev);
    if (prev != dev) hipSetDevice(dev);
  }
  ~DevGuard() {
    int cur = -1;
    hipGetDevice(&cur);
    if (prev >= 0 && cur != prev) hipSetDevice(prev);
  }
};

struct DBuf {                      // device scratch, grown on demand, on the current device
  void *p = nullptr;
  size_t bytes = 0;
  int dev = -1;
  hipError_t reserve(size_t n) {
    int cur = -1;
    hipGetDevice(&cur);
    if (n <= bytes && p && cur == dev) return hipSuccess;
    release();                     // too small, or allocated on another device
    n = std::max<size_t>(n, 64);
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) { bytes = n; hipGetDevice(&dev); }
    return e;
  }
  void release() {
    if (p) { DevGuard g(dev); hipFree(p); }
    p = nullptr;
    bytes = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
  ~DBuf() { release(); }
};

struct HBuf {                      // pinned host scratch
  void *p = nullptr;
  size_t bytes = 0;
  hipError_t reserve(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    if (p) { hipHostFree(p); p = nullptr; bytes = 0; }
    n = std::max<size_t>(n, 64);
    hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
    if (e == hipSuccess) bytes = n;
    return e;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
  ~HBuf() { if (p) hipHostFree(p); }
};

// ---------------------------------------------------------------------------
// transports

struct Transport {
  virtual ~Transport() {}
  virtual int kind() const = 0;                 // TFIDF_TRANSPORT_*
  virtual bool device_memory() const = 0;       // buffers are device memory (else host)
  virtual int all_gather(const void *send, void *recv, uint64_t bytes, hipStream_t s) = 0;
  virtual int all_to_all_v(const void *send, const uint64_t *sb, const uint64_t *so, void *recv, const uint64_t *rb,
                           const uint64_t *ro, hipStream_t s) = 0;
};

struct CallbackTransport : Transport {
  tfidf_collectives c;
  explicit CallbackTransport(const tfidf_collectives &x) : c(x) {}
  int kind() const override { return TFIDF_TRANSPORT_CALLBACK; }
  bool device_memory() const override { return c.memory == TFIDF_COLL_DEVICE; }
  int all_gather(const void *send, void *recv, uint64_t bytes, hipStream_t s) override {
    const int rc = c.all_gather(c.ctx, send, recv, bytes, (void *)s);
    return rc ? errf(TFIDF_E_HIP, "all_gather callback failed (%d)", rc) : TFIDF_OK;
  }
  int all_to_all_v(const void *send, const uint64_t *sb, const uint64_t *so, void *recv, const uint64_t *rb,
                   const uint64_t *ro, hipStream_t s) override {
    const int rc = c.all_to_all_v(c.ctx, send, sb, so, recv, rb, ro, (void *)s);
    return rc ? errf(TFIDF_E_HIP, "all_to_all_v callback failed (%d)", rc) : TFIDF_OK;
  }
};

// RCCL entry points, resolved from the librccl that sits next to the HIP
// runtime this library is bound to (a process with PyTorch loaded first runs
// the library on torch's runtime, whose directory holds its own librccl; a
// second RCCL bound to another runtime would not understand our streams).
struct RcclApi {
  bool ok = false;
  std::string err, path;
  ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

RcclApi &rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    std::vector<std::string> cand;
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(static_cast<hipError_t (*)(hipStream_t)>(&hipStreamSynchronize)), &info) && info.dli_fname) {
      std::string dir(info.dli_fname);
      const size_t sl = dir.rfind('/');
      dir = sl == std::string::npos ? std::string(".") : dir.substr(0, sl);
      cand.push_back(dir + "/librccl.so.1");
      cand.push_back(dir + "/librccl.so");
    }
    cand.push_back("/opt/rocm/lib/librccl.so.1");
    void *h = nullptr;
    for (const std::string &c : cand) {
      h = dlopen(c.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (h) { api.path = c; break; }
    }
    if (!h) { api.err = std::string("librccl not found next to the HIP runtime: ") + dlerror(); return; }
    bool all = true;
    auto sym = [&](auto &fp, const char *name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      all &= fp != nullptr;
    };
    sym(api.GetUniqueId, "ncclGetUniqueId");
    sym(api.CommInitRank, "ncclCommInitRank");
    sym(api.CommInitAll, "ncclCommInitAll");
    sym(api.CommDestroy, "ncclCommDestroy");
    sym(api.AllGather, "ncclAllGather");
    sym(api.Send, "ncclSend");
    sym(api.Recv, "ncclRecv");
    sym(api.GroupStart, "ncclGroupStart");
    sym(api.GroupEnd, "ncclGroupEnd");
    sym(api.GetErrorString, "ncclGetErrorString");
    if (!all) { api.err = "librccl lacks an entry point (" + api.path + ")"; return; }
    api.ok = true;
  });
  return api;
}

#define NCCL_TRY(expr)                                                                              \
  do {                                                                                              \
    ncclResult_t _r = (expr);                                                                       \
    if (_r != ncclSuccess) return errf(TFIDF_E_HIP, "%s: %s", #expr, rccl().GetErrorString(_r));    \
  } while (0)

struct RcclTransport : Transport {
  ncclComm_t comm = nullptr;
  int world = 1;
  RcclTransport(ncclComm_t c, int w) : comm(c), world(w) {}
  ~RcclTransport() override {
    if (comm) rccl().CommDestroy(comm);
  }
  int kind() const override { return TFIDF_TRANSPORT_RCCL; }
  bool device_memory() const override { return true; }
  int all_gather(const void *send, void *recv, uint64_t bytes, hipStream_t s) override {
    NCCL_TRY(rccl().AllGather(send, recv, bytes, ncclUint8, comm, s));
    return TFIDF_OK;
  }
  int all_to_all_v(const void *send, const uint64_t *sb, const uint64_t *so, void *recv, const uint64_t *rb,
                   const uint64_t *ro, hipStream_t s) override {
    // point-to-point pairs in one group: every xGMI link carries its own pair
    NCCL_TRY(rccl().GroupStart());
    for (int r = 0; r < world; r++) {
      if (sb[r]) NCCL_TRY(rccl().Send(static_cast<const uint8_t *>(send) + so[r], sb[r], ncclUint8, r, comm, s));
      if (rb[r]) NCCL_TRY(rccl().Recv(static_cast<uint8_t *>(recv) + ro[r], rb[r], ncclUint8, r, comm, s));
    }
    NCCL_TRY(rccl().GroupEnd());
    return TFIDF_OK;
  }
};

// Shards of one process exchanging through host memory (tfidf_node with a
// repeated device, or TFIDF_NODE_INPROC): a generation barrier around each
// exchange; each rank copies what it receives from the senders' buffers.
struct InprocGroup {
  int world;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t phase = 0;
  int arrived = 0;
  std::vector<const void *> sp;
  std::vector<const uint64_t *> sb, so;
  explicit InprocGroup(int w) : world(w), sp(w), sb(w), so(w) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t my = phase;
    if (++arrived == world) {
      arrived = 0;
      phase++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return phase != my; });
    }
  }
};

struct InprocTransport : Transport {
  std::shared_ptr<InprocGroup> g;
  int rank;
  InprocTransport(std::shared_ptr<InprocGroup> grp, int r) : g(std::move(grp)), rank(r) {}
  int kind() const override { return TFIDF_TRANSPORT_INPROC; }
  bool device_memory() const override { return false; }
  int all_gather(const void *send, void *recv, uint64_t bytes, hipStream_t) override {
    g->sp[rank] = send;
    g->barrier();
    for (int r = 0; r < g->world; r++)
      if (bytes) memcpy(static_cast<uint8_t *>(recv) + (size_t)r * bytes, g->sp[r], bytes);
    g->barrier();                                   // senders' buffers are free again
    return TFIDF_OK;
  }
  int all_to_all_v(const void *send, const uint64_t *sb, const uint64_t *so, void *recv, const uint64_t *rb,
                   const uint64_t *ro, hipStream_t) override {
    g->sp[rank] = send;
    g->sb[rank] = sb;
    g->so[rank] = so;
    g->barrier();
    int bad = -1;
    for (int r = 0; r < g->world; r++) {
      const uint64_t n = g->sb[r][rank];
      if (n != rb[r]) bad = r;
      else if (n) memcpy(static_cast<uint8_t *>(recv) + ro[r], static_cast<const uint8_t *>(g->sp[r]) + g->so[r][rank], n);
    }
    g->barrier();
    return bad >= 0 ? errf(TFIDF_E_INVALID_ARG, "all_to_all_v: rank %d sends a different size than rank %d expects",
                           bad, rank)
                    : TFIDF_OK;
  }
};

}  // namespace

// ---------------------------------------------------------------------------
// communicator: a transport + this rank's scratch and last results

struct tfidf_comm {
  int rank = 0, world = 1;
  int device = -1;                  // the communicator's GPU (RCCL), -1: the caller's current device
  std::unique_ptr<Transport> t;
  // staging between the transport's memory and the other kind
  DBuf d_stage_in, d_stage_out;
  HBuf h_stage_in, h_stage_out;
  // orchestration scratch (device)
  DBuf d_rec, d_cnt, d_got, d_ans, d_back, d_nu, d_keys, d_all, d_out, d_srt_k, d_srt_v, d_seg, d_tmp;
  HBuf h_out;
  // SHARD mode name table (tfidf_dist_shard_commit): every rank's names,
  // sorted by String.compareTo, distinct; this rank's doc -> name id
  std::string names;
  std::vector<uint64_t> name_off{0};
  DBuf d_name_of_doc;
  uint64_t names_gen = ~0ull;       // index commit generation the name table was built for
  bool names_ready = false;
  uint64_t global_gen = ~0ull;      // index commit generation of the last GLOBAL exchange
  uint64_t last_failed = 0;         // SHARD search: ranks skipped by the last search (bit r)
  HBuf h_hdr;                       // status words ahead of a rank's keys (pinned)
  DBuf d_meta, d_M;                 // GLOBAL exchange: this rank's meta row / every rank's (device)
  HBuf h_meta, h_M;                 // their pinned host sides
  bool hdr_pending = false;         // an upload out of h_hdr may still be queued (a search that failed)
  // last search results (tfidf_dist_last_hits / _last_names)
  std::vector<uint64_t> last_doc;
  std::vector<float> last_score;
  std::vector<uint32_t> last_name;
  std::vector<double> last_sum;
  uint64_t last_name_bytes = 0;
};

namespace {

// gather `bytes` per rank: src / dst are device buffers (dev) or host buffers
int coll_gather(tfidf_comm *c, hipStream_t s, const void *src, void *dst, uint64_t bytes, bool dev) {
  const uint64_t tot = bytes * (uint64_t)c->world;
  if (bytes == 0) return TFIDF_OK;                        // every rank knows: no call
  if (c->t->device_memory() == dev) {
    if (dev) return c->t->all_gather(src, dst, bytes, s);
    return c->t->all_gather(src, dst, bytes, nullptr);
  }
  if (dev) {                                              // device data over a host transport
    DHIP(c->h_stage_in.reserve(bytes));
    DHIP(c->h_stage_out.reserve(tot));
    DHIP(hipMemcpyAsync(c->h_stage_in.p, src, bytes, hipMemcpyDeviceToHost, s));
    DHIP(hipStreamSynchronize(s));
    if (int rc = c->t->all_gather(c->h_stage_in.p, c->h_stage_out.p, bytes, nullptr)) return rc;
    DHIP(hipMemcpyAsync(dst, c->h_stage_out.p, tot, hipMemcpyHostToDevice, s));
    return TFIDF_OK;
  }
  // host data over a device transport
  DHIP(c->d_stage_in.reserve(bytes));
  DHIP(c->d_stage_out.reserve(tot));
  DHIP(hipMemcpyAsync(c->d_stage_in.p, src, bytes, hipMemcpyHostToDevice, s));
  if (int rc = c->t->all_gather(c->d_stage_in.p, c->d_stage_out.p, bytes, s)) return rc;
  DHIP(hipMemcpyAsync(dst, c->d_stage_out.p, tot, hipMemcpyDeviceToHost, s));
  DHIP(hipStreamSynchronize(s));
  return TFIDF_OK;
}

int coll_a2av(tfidf_comm *c, hipStream_t s, const void *src, const uint64_t *sb, const uint64_t *so, void *dst,
              const uint64_t *rb, const uint64_t *ro, bool dev) {
  uint64_t send_tot = 0, recv_tot = 0;
  for (int r = 0; r < c->world; r++) {
    send_tot = std::max(send_tot, so[r] + sb[r]);
    recv_tot = std::max(recv_tot, ro[r] + rb[r]);
  }
  if (c->t->device_memory() == dev) return c->t->all_to_all_v(src, sb, so, dst, rb, ro, dev ? s : nullptr);
  if (dev) {
    DHIP(c->h_stage_in.reserve(send_tot));
    DHIP(c->h_stage_out.reserve(recv_tot));
    if (send_tot) DHIP(hipMemcpyAsync(c->h_stage_in.p, src, send_tot, hipMemcpyDeviceToHost, s));
    DHIP(hipStreamSynchronize(s));
    if (int rc = c->t->all_to_all_v(c->h_stage_in.p, sb, so, c->h_stage_out.p, rb, ro, nullptr)) return rc;
    if (recv_tot) DHIP(hipMemcpyAsync(dst, c->h_stage_out.p, recv_tot, hipMemcpyHostToDevice, s));
    return TFIDF_OK;
  }
  DHIP(c->d_stage_in.reserve(send_tot));
  DHIP(c->d_stage_out.reserve(recv_tot));
  if (send_tot) DHIP(hipMemcpyAsync(c->d_stage_in.p, src, send_tot, hipMemcpyHostToDevice, s));
  if (int rc = c->t->all_to_all_v(c->d_stage_in.p, sb, so, c->d_stage_out.p, rb, ro, s)) return rc;
  if (recv_tot) DHIP(hipMemcpyAsync(dst, c->d_stage_out.p, recv_tot, hipMemcpyDeviceToHost, s));
  DHIP(hipStreamSynchronize(s));
  return TFIDF_OK;
}

// host all-gather of one u64 row per rank -> rows[world][n]
int gather_rows(tfidf_comm *c, hipStream_t s, const std::vector<uint64_t> &mine, std::vector<uint64_t> *rows) {
  rows->assign((size_t)c->world * mine.size(), 0);
  return coll_gather(c, s, mine.data(), rows->data(), mine.size() * 8, false);
}

// ---------------------------------------------------------------------------
// device kernels of the merges

// One thread per candidate key: its rank among the keys of every list of its
// query = its index in its own list + the keys above it in the others (lists
// are sorted descending; keys are distinct: global doc ids differ), found by
// binary search.  Candidates ranked below k_out are written at their rank.
__global__ void __launch_bounds__(256) k_merge_lists(const uint64_t *keys, uint32_t n_lists, uint64_t rstride,
                                                     uint64_t qstride, uint64_t len, uint32_t n_q, uint64_t *out,
                                                     uint64_t k_out) {
  const uint64_t per_q = (uint64_t)n_lists * len;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per_q * n_q) return;
  const uint32_t q = (uint32_t)(t / per_q);
  const uint64_t rem = t - (uint64_t)q * per_q;
  const uint32_t r = (uint32_t)(rem / len);
  const uint64_t i = rem - (uint64_t)r * len;
  const uint64_t x = keys[(uint64_t)r * rstride + (uint64_t)q * qstride + i];
  if (x == 0 || i >= k_out) return;
  uint64_t rank = i;
  for (uint32_t o = 0; o < n_lists && rank < k_out; o++) {
    if (o == r) continue;
    const uint64_t *l = keys + (uint64_t)o * rstride + (uint64_t)q * qstride;
    uint64_t a = 0, z = len;                    // first index whose key is < x (keys above x: [0, a))
    while (a < z) {
      const uint64_t m = (a + z) >> 1;
      if (l[m] > x) a = m + 1; else z = m;
    }
    rank += a;
  }
  if (rank < k_out) out[(uint64_t)q * k_out + rank] = x;
}

// SHARD mode: (name id << 32 | score bits) records of every hit key (local doc ids)
__global__ void k_name_records(const uint64_t *keys, uint64_t n, const uint32_t *name_of_doc, uint64_t *rec) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = keys[i];
  const uint32_t doc = ~(uint32_t)k;
  rec[i] = ((uint64_t)name_of_doc[doc] << 32) | (k >> 32);
}

// gathered [world][maxn] records (rows padded) -> key (name id) / value (score bits) arrays in rank order
__global__ void k_split_records(const uint64_t *all, uint64_t maxn, const uint64_t *row_n, const uint64_t *row_base,
                                uint32_t world, uint32_t *kk, uint32_t *vv) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= maxn * world) return;
  const uint32_t r = (uint32_t)(t / maxn);
  const uint64_t i = t - (uint64_t)r * maxn;
  if (i >= row_n[r]) return;
  const uint64_t x = all[t];
  kk[row_base[r] + i] = (uint32_t)(x >> 32);
  vv[row_base[r] + i] = (uint32_t)x;
}

__global__ void k_seg_heads(const uint32_t *k, uint64_t n, uint32_t *head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) head[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
}

// Per name, the scores ((double) of each float) summed in rank order
// (HashMap.merge with Double::sum in worker-response order, Leader.java:73-77):
// the stable sort kept that order inside each name's run.
__global__ void k_seg_sums(const uint32_t *k, const uint32_t *v, const uint32_t *pos, uint64_t n, uint32_t *out_name,
                           double *out_sum) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (i > 0 && k[i] == k[i - 1])) return;
  double s = (double)__uint_as_float(v[i]);
  for (uint64_t j = i + 1; j < n && k[j] == k[i]; j++) s += (double)__uint_as_float(v[j]);
  out_name[pos[i]] = k[i];
  out_sum[pos[i]] = s;
}

inline unsigned grid_of(uint64_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

hipError_t tfidf::launch_merge_lists(const uint64_t *keys, uint32_t n_lists, uint64_t rstride, uint64_t qstride,
                                     uint64_t len, uint32_t n_q, uint64_t *out, uint64_t k_out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, (size_t)n_q * k_out * 8, s);
  if (e != hipSuccess) return e;
  const uint64_t n = (uint64_t)n_q * n_lists * len;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_merge_lists, dim3(grid_of(n)), dim3(256), 0, s, keys, n_lists, rstride, qstride, len, n_q, out,
                     k_out);
  return hipGetLastError();
}

namespace {

void decode_keys(const uint64_t *k, uint64_t n, uint64_t *doc, float *score) {
  for (uint64_t i = 0; i < n; i++) {
    doc[i] = (~k[i]) & 0xFFFFFFFFull;
    const uint32_t b = (uint32_t)(k[i] >> 32);
    memcpy(&score[i], &b, 4);
  }
}

// the query status every rank computes alike (no collective when it fails)
int query_status(const uint8_t *q, uint64_t n) {
  QueryPlan plan;
  const int rc = parse_query(q, n, &plan);
  if (rc == kQBadUtf8) return errf(TFIDF_E_UNSUPPORTED_QUERY, "query is not valid UTF-8");
  if (rc == kQSyntax) return errf(TFIDF_E_QUERY_SYNTAX, "query does not parse (QueryParser ParseException / TooManyClauses)");
  return TFIDF_OK;
}

int check_comm(tfidf_index *ix, tfidf_comm *c) {
  if (!ix || !c) return errf(TFIDF_E_INVALID_ARG, "NULL index or communicator");
  return TFIDF_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// communicators

extern "C" int tfidf_comm_create(int32_t rank, int32_t world, const tfidf_collectives *coll, tfidf_comm **out) {
  if (!coll || !out || !coll->all_gather || !coll->all_to_all_v) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  if (world < 1 || rank < 0 || rank >= world) return errf(TFIDF_E_INVALID_ARG, "rank %d / world %d", rank, world);
  if (coll->memory != TFIDF_COLL_HOST && coll->memory != TFIDF_COLL_DEVICE)
    return errf(TFIDF_E_INVALID_ARG, "memory must be TFIDF_COLL_HOST or TFIDF_COLL_DEVICE");
  tfidf_comm *c = new tfidf_comm();
  c->rank = rank;
  c->world = world;
  c->t.reset(new CallbackTransport(*coll));
  *out = c;
  return TFIDF_OK;
}

extern "C" int tfidf_rccl_unique_id(uint8_t id[128]) {
  if (!id) return errf(TFIDF_E_INVALID_ARG, "NULL id");
  RcclApi &api = rccl();
  if (!api.ok) return errf(TFIDF_E_NO_DEVICE, "%s", api.err.c_str());
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId u;
  NCCL_TRY(api.GetUniqueId(&u));
  memcpy(id, &u, 128);
  return TFIDF_OK;
}

extern "C" int tfidf_comm_init_rccl(const uint8_t id[128], int32_t rank, int32_t world, int32_t device,
                                    tfidf_comm **out) {
  if (!id || !out) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  if (world < 1 || rank < 0 || rank >= world) return errf(TFIDF_E_INVALID_ARG, "rank %d / world %d", rank, world);
  RcclApi &api = rccl();
  if (!api.ok) return errf(TFIDF_E_NO_DEVICE, "%s", api.err.c_str());
  DevGuard g(device);
  ncclUniqueId u;
  memcpy(&u, id, 128);
  ncclComm_t comm = nullptr;
  NCCL_TRY(api.CommInitRank(&comm, world, u, rank));
  tfidf_comm *c = new tfidf_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  c->t.reset(new RcclTransport(comm, world));
  *out = c;
  return TFIDF_OK;
}

extern "C" int tfidf_comm_create_inproc(int32_t world, tfidf_comm **comms) {
  if (!comms || world < 1 || world > 1024) return errf(TFIDF_E_INVALID_ARG, "NULL comms or world out of range");
  auto grp = std::make_shared<InprocGroup>(world);
  for (int32_t i = 0; i < world; i++) {
    tfidf_comm *c = new tfidf_comm();
    c->rank = i;
    c->world = world;
    c->t.reset(new InprocTransport(grp, i));
    comms[i] = c;
  }
  return TFIDF_OK;
}

extern "C" int tfidf_comm_destroy(tfidf_comm *c) {
  delete c;
  return TFIDF_OK;
}

extern "C" int tfidf_comm_info(const tfidf_comm *c, int32_t *rank, int32_t *world, int32_t *transport) {
  if (!c) return errf(TFIDF_E_INVALID_ARG, "NULL communicator");
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  if (transport) *transport = c->t->kind();
  return TFIDF_OK;
}

extern "C" int tfidf_comm_selftest(tfidf_comm *c) {
  if (!c) return errf(TFIDF_E_INVALID_ARG, "NULL communicator");
  const int ws = c->world, me = c->rank;
  int cur = 0;
  hipGetDevice(&cur);
  DevGuard g(c->device >= 0 ? c->device : cur);      // staging buffers on the communicator's GPU
  hipStream_t s = nullptr;                            // (the null stream of that device)
  // all-gather of (rank, world) rows
  std::vector<uint64_t> rows;
  if (int rc = gather_rows(c, s, {(uint64_t)me, (uint64_t)ws, 0xC0FFEEull}, &rows)) return rc;
  for (int r = 0; r < ws; r++)
    if (rows[3 * r] != (uint64_t)r || rows[3 * r + 1] != (uint64_t)ws || rows[3 * r + 2] != 0xC0FFEEull)
      return errf(TFIDF_E_HIP, "selftest: all_gather row %d wrong", r);
  // all-to-all-v: rank me sends (me + 1) * (r + 1) bytes of value (me * 16 + r) & 0xFF to rank r
  std::vector<uint64_t> sb(ws), so(ws), rb(ws), ro(ws);
  uint64_t st = 0, rt = 0;
  for (int r = 0; r < ws; r++) {
    sb[r] = (uint64_t)(me + 1) * (r + 1);
    so[r] = st;
    st += sb[r];
    rb[r] = (uint64_t)(r + 1) * (me + 1);
    ro[r] = rt;
    rt += rb[r];
  }
  std::vector<uint8_t> snd(st), rcv(rt, 0xEE);
  for (int r = 0; r < ws; r++) memset(snd.data() + so[r], (me * 16 + r) & 0xFF, sb[r]);
  if (int rc = coll_a2av(c, s, snd.data(), sb.data(), so.data(), rcv.data(), rb.data(), ro.data(), false)) return rc;
  for (int r = 0; r < ws; r++)
    for (uint64_t i = 0; i < rb[r]; i++)
      if (rcv[ro[r] + i] != (uint8_t)((r * 16 + me) & 0xFF))
        return errf(TFIDF_E_HIP, "selftest: all_to_all_v bytes from rank %d wrong", r);
  return TFIDF_OK;
}

// ---------------------------------------------------------------------------
// process model (2): per-rank orchestration

// GLOBAL statistics by term ownership.  Meta row per rank: [records per owner
// (world) | docCount | sumTTF | seed attempt | error] — one host read; the
// ranks see each other's errors and seed attempts in it, so they fail, or
// re-commit under one seed, together.  Round 6: one host synchronisation per
// exchange (the gathered meta rows): the owner counts stay on the device
// (written by the partition straight into the meta row), the partition,
// reduction and df import queue without waiting, and the new statistics view
// is published behind an event the first search waits for.
extern "C" int tfidf_dist_global_commit(tfidf_index *ix, tfidf_comm *c, uint64_t *n_vocab, uint64_t *doc_count,
                                        uint64_t *sum_ttf) {
  if (int rc = check_comm(ix, c)) return rc;
  const int ws = c->world, me = c->rank;
  const size_t W = ws + 4;
  DevGuard g(index_device(ix));
  hipStream_t s = index_stream(ix);
  int local_err = index_committed(ix) ? TFIDF_OK : errf(TFIDF_E_STATE, "index not committed");
  std::string local_msg = local_err ? tfidf_last_error() : "";
  DHIP(c->d_meta.reserve(W * 8));
  DHIP(c->d_M.reserve((size_t)ws * W * 8));
  DHIP(c->h_meta.reserve(W * 8));
  DHIP(c->h_M.reserve((size_t)ws * W * 8));
  uint64_t *meta = c->h_meta.as<uint64_t>();
  const uint64_t *M = c->h_M.as<uint64_t>();
  uint64_t n_rec = 0;
  for (int round = 0;; round++) {
    tfidf_index_stats st{};
    if (!local_err) local_err = tfidf_stats(ix, &st);
    if (!local_err) {
      DHIP(c->d_rec.reserve(std::max<uint64_t>(st.num_terms, 1) * 24));
      local_err = vocab_partition_async(ix, (uint32_t)ws, c->d_rec.p, c->d_rec.bytes / 24, c->d_meta.p, &n_rec);
    }
    if (local_err && local_msg.empty()) local_msg = tfidf_last_error();
    if (local_err) DHIP(hipMemsetAsync(c->d_meta.p, 0, (size_t)ws * 8, s));
    meta[ws] = st.doc_count;
    meta[ws + 1] = st.sum_ttf;
    meta[ws + 2] = st.hash_rebuilds;
    meta[ws + 3] = local_err ? (uint64_t)local_err : 0;
    DHIP(hipMemcpyAsync(c->d_meta.as<uint64_t>() + ws, meta + ws, 4 * 8, hipMemcpyHostToDevice, s));
    if (int rc = coll_gather(c, s, c->d_meta.p, c->d_M.p, W * 8, true)) return rc;
    DHIP(hipMemcpyAsync(c->h_M.p, c->d_M.p, (size_t)ws * W * 8, hipMemcpyDeviceToHost, s));
    DHIP(hipStreamSynchronize(s));                    // the one host read (meta rows; h_meta reusable)
    for (int r = 0; r < ws; r++)
      if (M[r * W + ws + 3]) {
        if (r == me) return set_error(local_err, local_msg.c_str());
        return errf((int)M[r * W + ws + 3], "rank %d failed in the GLOBAL statistics exchange", r);
      }
    uint64_t top = 0;
    bool same = true;
    for (int r = 0; r < ws; r++) top = std::max(top, M[r * W + ws + 2]);
    for (int r = 0; r < ws; r++) same &= M[r * W + ws + 2] == top;
    if (same) break;
    if (round > 8) return errf(TFIDF_E_STATE, "hash seed agreement did not converge");
    // a shard met a hash collision and rebuilt under a later seed: keys are
    // matched across shards, so the shards below it re-commit under that
    // seed (which may collide there in turn: agree again next round)
    if (st.hash_rebuilds < top) {
      local_err = tfidf_set_hash_attempt(ix, (uint32_t)top);
      if (!local_err) local_err = tfidf_commit(ix);
      tfidf_set_hash_attempt(ix, 0);
      if (local_err) local_msg = tfidf_last_error();
    }
  }
  std::vector<uint64_t> sb(ws), so(ws), rb(ws), ro(ws), sb2(ws), so2(ws), rb2(ws), ro2(ws);
  uint64_t gdc = 0, gttf = 0, n_got = 0, at = 0, at2 = 0;
  for (int r = 0; r < ws; r++) {
    gdc += M[r * W + ws];
    gttf += M[r * W + ws + 1];
    sb[r] = M[me * W + r] * 24;
    so[r] = at;
    at += sb[r];
    rb[r] = M[r * W + me] * 24;
    ro[r] = n_got * 24;
    n_got += M[r * W + me];
    // answers travel back: one u32 per record
    sb2[r] = M[r * W + me] * 4;
    so2[r] = ro[r] / 6;
    rb2[r] = M[me * W + r] * 4;
    ro2[r] = at2;
    at2 += rb2[r];
  }
  DHIP(c->d_got.reserve(std::max<uint64_t>(n_got, 1) * 24));
  if (int rc = coll_a2av(c, s, c->d_rec.p, sb.data(), so.data(), c->d_got.p, rb.data(), ro.data(), true)) return rc;
  DHIP(c->d_ans.reserve(std::max<uint64_t>(n_got, 1) * 4));
  DHIP(c->d_nu.reserve(8));
  if (int rc = vocab_reduce_async(ix, c->d_got.p, n_got, c->d_ans.p, c->d_nu.p)) return rc;
  DHIP(c->d_back.reserve(std::max<uint64_t>(n_rec, 1) * 4));
  if (int rc = coll_a2av(c, s, c->d_ans.p, sb2.data(), so2.data(), c->d_back.p, rb2.data(), ro2.data(), true)) return rc;
  // the generation the view was published on (not re-read: a commit on another
  // thread may have landed since)
  uint64_t gen = 0;
  if (int rc = set_global_df_async(ix, c->d_back.p, n_rec, gdc, gttf, &gen)) return rc;
  c->global_gen = gen;
  if (n_vocab) {
    uint64_t nu = 0;
    DHIP(hipMemcpyAsync(&nu, c->d_nu.p, 8, hipMemcpyDeviceToHost, s));
    DHIP(hipStreamSynchronize(s));
    std::vector<uint64_t> rows;
    if (int rc = gather_rows(c, s, {nu}, &rows)) return rc;
    uint64_t tot = 0;
    for (uint64_t x : rows) tot += x;
    *n_vocab = tot;
  }
  if (doc_count) *doc_count = gdc;
  if (sum_ttf) *sum_ttf = gttf;
  return TFIDF_OK;
}

namespace {

// ---- search-time agreement (round-4 advisor finding).  Every rank's local
// status travels in the first collective of a search — as a header ahead of
// its top-k keys, or in the count row of a variable-length gather — so a rank
// that cannot serve (index not committed, re-committed since the last GLOBAL
// exchange or name table, doc range past 2^32, a failed local search) never
// leaves the others waiting in the data collective: GLOBAL searches then fail
// on every rank together; SHARD searches merge the healthy ranks' hits
// (Leader.start skips a failed worker, Leader.java:67-69).  The header also
// carries (doc_base, n_docs): GLOBAL merge keys must not collide, so
// overlapping doc ranges fail on every rank (TFIDF_E_INVALID_ARG).
constexpr uint64_t kHdr = 4;        // status words per rank: {rc, doc_base, n_docs, 0}

// One snapshot for a whole node-level search: the status check,
// the local search and the document count all read the reader it pins, so a
// commit landing on another thread meanwhile cannot mix generations.
struct Pinned {
  tfidf_reader *rd = nullptr;
  uint64_t gen = 0, nd = 0;
  Pinned() = default;
  Pinned(const Pinned &) = delete;
  Pinned &operator=(const Pinned &) = delete;
  ~Pinned() { if (rd) tfidf_reader_close(rd); }
  int open(tfidf_index *ix) {
    if (tfidf_reader_open(ix, &rd) != TFIDF_OK) { rd = nullptr; return errf(TFIDF_E_STATE, "index not committed"); }
    return tfidf_reader_info(rd, &gen, &nd);
  }
};

int local_search_status(Pinned &pin, tfidf_index *ix, tfidf_comm *c, uint64_t doc_base, bool global) {
  if (int rc = pin.open(ix)) return rc;
  if (doc_base + pin.nd > (1ull << 32))
    return errf(TFIDF_E_CAPACITY, "global doc ids must stay below 2^32 (merge keys carry 32-bit ids)");
  if (global && c->global_gen != pin.gen)
    return errf(TFIDF_E_STATE, "tfidf_dist_global_commit first (after every commit)");
  if (!global && (!c->names_ready || c->names_gen != pin.gen))
    return errf(TFIDF_E_STATE, "tfidf_dist_shard_commit first (after every commit)");
  return TFIDF_OK;
}

// Verdict over every rank's status words (rows of `stride` u64: rc, base, n):
// the first failing rank's error (its own message on that rank); GLOBAL mode
// also checks that the doc ranges do not overlap.  *failed = mask of failing ranks.
int status_verdict(tfidf_comm *c, const uint64_t *rows, size_t stride, int lrc, const std::string &lmsg,
                   bool fail_together, uint64_t *failed) {
  const int ws = c->world;
  uint64_t mask = 0;
  int first = -1;
  for (int r = 0; r < ws; r++)
    if (rows[(size_t)r * stride]) {
      if (r < 64) mask |= 1ull << r;
      if (first < 0) first = r;
    }
  if (failed) *failed = mask;
  if (first >= 0 && fail_together) {
    if (first == c->rank) return set_error(lrc, lmsg.c_str());
    return errf((int)rows[(size_t)first * stride], "rank %d cannot serve the search", first);
  }
  if (fail_together) {
    std::vector<std::pair<uint64_t, uint64_t>> rg;
    for (int r = 0; r < ws; r++)
      if (rows[(size_t)r * stride + 2]) rg.emplace_back(rows[(size_t)r * stride + 1], rows[(size_t)r * stride + 2]);
    std::sort(rg.begin(), rg.end());
    for (size_t i = 1; i < rg.size(); i++)
      if (rg[i - 1].first + rg[i - 1].second > rg[i].first)
        return errf(TFIDF_E_INVALID_ARG, "shard doc ranges overlap ([%llu, +%llu) and [%llu, +%llu))",
                    (unsigned long long)rg[i - 1].first, (unsigned long long)rg[i - 1].second,
                    (unsigned long long)rg[i].first, (unsigned long long)rg[i].second);
  }
  return TFIDF_OK;
}

int write_hits(tfidf_comm *c, uint64_t *doc_ids, float *scores, uint64_t cap, uint64_t *n_out) {
  const uint64_t n = c->last_doc.size();
  *n_out = n;
  const uint64_t m = std::min(n, cap);
  if (m && doc_ids) memcpy(doc_ids, c->last_doc.data(), m * 8);
  if (m && scores) memcpy(scores, c->last_score.data(), m * 4);
  if (n > cap) return errf(TFIDF_E_BUFFER, "%llu hits (tfidf_dist_last_hits holds them)", (unsigned long long)n);
  return TFIDF_OK;
}

// every hit's merge key of one query on this shard -> d_keys; *h = hits
int all_keys(Pinned &pin, tfidf_comm *c, const uint8_t *q, uint64_t q_len, uint64_t doc_base, uint64_t *h) {
  const uint64_t nd = std::max<uint64_t>(pin.nd, 1);
  DHIP(c->d_keys.reserve(nd * 8));
  return reader_all_keys_device(pin.rd, q, q_len, doc_base, c->d_keys.p, nd, h);
}

// gather variable-length device rows (d_keys[0, h)) from every rank, padded to
// the longest with `pad` -> d_all [world][maxn]; ns = every rank's count.  The
// count row carries the rank's status first (a failing rank sends h = 0).
int gather_var(tfidf_comm *c, hipStream_t s, uint64_t h, uint64_t pad_byte, int lrc, const std::string &lmsg,
               uint64_t doc_base, uint64_t n_docs, bool fail_together, std::vector<uint64_t> *ns, uint64_t *maxn) {
  if (lrc) h = 0;
  std::vector<uint64_t> rows;
  if (int rc = gather_rows(c, s, {(uint64_t)lrc, doc_base, n_docs, h}, &rows)) return rc;
  if (int rc = status_verdict(c, rows.data(), 4, lrc, lmsg, fail_together, &c->last_failed)) return rc;
  ns->assign(c->world, 0);
  uint64_t mx = 0;
  for (int r = 0; r < c->world; r++) {
    (*ns)[r] = rows[(size_t)r * 4 + 3];
    mx = std::max(mx, (*ns)[r]);
  }
  *maxn = mx;
  if (mx == 0) return TFIDF_OK;
  DHIP(c->d_out.reserve(mx * 8));
  if (h) DHIP(hipMemcpyAsync(c->d_out.p, c->d_keys.p, h * 8, hipMemcpyDeviceToDevice, s));
  if (mx > h) DHIP(hipMemsetAsync(c->d_out.as<uint64_t>() + h, (int)pad_byte, (mx - h) * 8, s));
  DHIP(c->d_all.reserve((size_t)c->world * mx * 8));
  return coll_gather(c, s, c->d_out.p, c->d_all.p, mx * 8, true);
}

// Top-k keys of this rank's n_q queries with the status header ahead of them
// (row = kHdr + n_q k words), all-gathered, merged per query on the device into
// d_out [n_q][k]; the merged keys and every rank's header are read back into
// h_out ([n_q k] keys, then [world][kHdr]).  A failing rank sends zero keys.
int gather_topk(tfidf_index *ix, tfidf_comm *c, hipStream_t s, uint64_t doc_base, const uint8_t *q_utf8,
                const uint64_t *q_offsets, uint32_t n_q, uint32_t k) {
  const int ws = c->world;
  const uint64_t per = (uint64_t)n_q * k, row = kHdr + per;
  DHIP(c->d_keys.reserve(row * 8));                    // only an allocation failure returns before the exchange
  DHIP(c->d_all.reserve((size_t)ws * row * 8));
  DHIP(c->d_out.reserve(per * 8));
  DHIP(c->h_out.reserve((per + (size_t)ws * kHdr) * 8));
  DHIP(c->h_hdr.reserve(kHdr * 8));
  uint64_t *dk = c->d_keys.as<uint64_t>();
  Pinned pin;
  int lrc = local_search_status(pin, ix, c, doc_base, true);
  if (!lrc) lrc = reader_batch_keys_device(pin.rd, q_utf8, q_offsets, n_q, k, doc_base, dk + kHdr);
  const std::string lmsg = lrc ? tfidf_last_error() : "";
  if (lrc) DHIP(hipMemsetAsync(dk + kHdr, 0, per * 8, s));
  uint64_t *hh = c->h_hdr.as<uint64_t>();
  if (c->hdr_pending) DHIP(hipStreamSynchronize(s));   // a failed search's header upload has left
  c->hdr_pending = true;
  hh[0] = (uint64_t)lrc;
  hh[1] = doc_base;
  hh[2] = lrc ? 0 : pin.nd;
  hh[3] = 0;
  DHIP(hipMemcpyAsync(dk, hh, kHdr * 8, hipMemcpyHostToDevice, s));
  if (int rc = coll_gather(c, s, dk, c->d_all.p, row * 8, true)) return rc;
  DHIP(launch_merge_lists(c->d_all.as<uint64_t>() + kHdr, (uint32_t)ws, row, k, k, n_q, c->d_out.as<uint64_t>(), k, s));
  uint64_t *ho = c->h_out.as<uint64_t>();
  DHIP(hipMemcpyAsync(ho, c->d_out.p, per * 8, hipMemcpyDeviceToHost, s));
  DHIP(hipMemcpy2DAsync(ho + per, kHdr * 8, c->d_all.p, row * 8, kHdr * 8, ws, hipMemcpyDeviceToHost, s));
  DHIP(hipStreamSynchronize(s));
  c->hdr_pending = false;
  return status_verdict(c, ho + per, kHdr, lrc, lmsg, true, nullptr);
}

}  // namespace

extern "C" int tfidf_dist_search(tfidf_index *ix, tfidf_comm *c, uint64_t doc_base, const uint8_t *q, uint64_t q_len,
                                 uint32_t k, uint64_t *doc_ids, float *scores, uint64_t cap, uint64_t *n_out) {
  if (int rc = check_comm(ix, c)) return rc;
  if (!n_out || (!q && q_len)) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  if (k > 1024) return errf(TFIDF_E_INVALID_ARG, "k must be <= 1024 (0 = all hits)");
  *n_out = 0;
  c->last_doc.clear();
  c->last_score.clear();
  if (int rc = query_status(q, q_len)) return rc;
  DevGuard g(index_device(ix));
  hipStream_t s = index_stream(ix);
  const int ws = c->world;
  uint64_t n = 0;
  if (k > 0) {
    const uint64_t offs[2] = {0, q_len};
    if (int rc = gather_topk(ix, c, s, doc_base, q, offs, 1, k)) return rc;
    const uint64_t *keys = c->h_out.as<uint64_t>();
    while (n < k && keys[n]) n++;
  } else {
    uint64_t h = 0, maxn = 0;
    Pinned pin;
    int lrc = local_search_status(pin, ix, c, doc_base, true);
    if (!lrc) lrc = all_keys(pin, c, q, q_len, doc_base, &h);
    const std::string lmsg = lrc ? tfidf_last_error() : "";
    std::vector<uint64_t> ns;
    if (int rc = gather_var(c, s, h, 0, lrc, lmsg, doc_base, lrc ? 0 : pin.nd, true, &ns, &maxn))
      return rc;
    for (uint64_t x : ns) n += x;
    if (n) {
      DHIP(c->d_tmp.reserve(n * 8));
      DHIP(launch_merge_lists(c->d_all.as<uint64_t>(), (uint32_t)ws, maxn, 0, maxn, 1, c->d_tmp.as<uint64_t>(), n, s));
      DHIP(c->h_out.reserve(n * 8));
      DHIP(hipMemcpyAsync(c->h_out.p, c->d_tmp.p, n * 8, hipMemcpyDeviceToHost, s));
      DHIP(hipStreamSynchronize(s));
    }
  }
  c->last_doc.resize(n);
  c->last_score.resize(n);
  decode_keys(c->h_out.as<uint64_t>(), n, c->last_doc.data(), c->last_score.data());
  return write_hits(c, doc_ids, scores, cap, n_out);
}

extern "C" int tfidf_dist_search_batch(tfidf_index *ix, tfidf_comm *c, uint64_t doc_base, const uint8_t *q_utf8,
                                       const uint64_t *q_offsets, uint32_t n_q, uint32_t k, uint64_t *doc_ids,
                                       float *scores, uint32_t *counts) {
  if (int rc = check_comm(ix, c)) return rc;
  if (!q_offsets || (n_q && (!doc_ids || !scores || !counts))) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  if (k == 0 || k > 1024) return errf(TFIDF_E_INVALID_ARG, "1 <= k <= 1024");
  if (n_q == 0) return TFIDF_OK;
  DevGuard g(index_device(ix));
  hipStream_t s = index_stream(ix);
  if (int rc = gather_topk(ix, c, s, doc_base, q_utf8, q_offsets, n_q, k)) return rc;
  const uint64_t *keys = c->h_out.as<uint64_t>();
  for (uint32_t i = 0; i < n_q; i++) {
    uint32_t m = 0;
    while (m < k && keys[(uint64_t)i * k + m]) m++;
    counts[i] = m;
    decode_keys(keys + (uint64_t)i * k, m, doc_ids + (uint64_t)i * k, scores + (uint64_t)i * k);
    for (uint32_t j = m; j < k; j++) {
      doc_ids[(uint64_t)i * k + j] = 0;
      scores[(uint64_t)i * k + j] = 0.0f;
    }
  }
  return TFIDF_OK;
}


namespace {
// SHARD search result with skipped ranks: TFIDF_OK (the healthy ranks' hits
// are the answer, as Leader.start returns the other workers' results), the
// skipped ranks in tfidf_dist_last_failed and, on every rank, a
// tfidf_last_error() message naming them (the failing rank's own reason there).
// When no rank could serve, every rank returns the (first) error instead.
int shard_partial(tfidf_comm *c, int lrc, const std::string &lmsg) {
  if (!c->last_failed) return TFIDF_OK;
  const int ws = std::min(c->world, 64);
  if (c->last_failed == (ws == 64 ? ~0ull : (1ull << ws) - 1)) {   // no rank answered: an error, not an empty map
    if (lrc) return set_error(lrc, lmsg.c_str());
    return errf(TFIDF_E_STATE, "no rank could serve the SHARD search");
  }
  std::string m = "SHARD search skipped rank(s)";
  for (int r = 0; r < c->world && r < 64; r++)
    if ((c->last_failed >> r) & 1u) m += " " + std::to_string(r);
  if (lrc) m += ": " + lmsg;
  set_error(lrc ? lrc : TFIDF_E_STATE, m.c_str());
  return TFIDF_OK;
}
}  // namespace

// SHARD mode name table: each rank sorts its own names (String.compareTo),
// the sorted lists are all-gathered and merged (distinct names in order);
// the rank's documents map to their name ids on the device.
extern "C" int tfidf_dist_shard_commit(tfidf_index *ix, tfidf_comm *c, uint64_t *n_names) {
  if (int rc = check_comm(ix, c)) return rc;
  const int ws = c->world, me = c->rank;
  DevGuard g(index_device(ix));
  hipStream_t s = index_stream(ix);
  c->names_ready = false;
  const uint64_t gen = index_generation(ix);
  int local_err = index_committed(ix) ? TFIDF_OK : errf(TFIDF_E_STATE, "index not committed");
  std::string local_msg = local_err ? tfidf_last_error() : "";
  const uint64_t nd = index_num_docs(ix);
  std::vector<uint64_t> offs(nd + 1, 0), perm(nd);
  std::string blob;
  if (!local_err) {
    uint64_t need = 0;
    int rc = tfidf_doc_keys(ix, nullptr, 0, offs.data(), &need);
    if (rc == TFIDF_OK || rc == TFIDF_E_BUFFER) {
      blob.resize(need);
      rc = tfidf_doc_keys(ix, reinterpret_cast<uint8_t *>(&blob[0]), need, offs.data(), &need);
    }
    if (!rc) rc = tfidf_sort_names(reinterpret_cast<const uint8_t *>(blob.data()), offs.data(), nd, perm.data());
    if (rc) { local_err = rc; local_msg = tfidf_last_error(); }
  }
  // sorted local names: lens + bytes
  std::vector<uint64_t> lens;
  std::string sorted;
  if (!local_err) {
    lens.resize(nd);
    sorted.reserve(blob.size());
    for (uint64_t i = 0; i < nd; i++) {
      const uint64_t d = perm[i];
      lens[i] = offs[d + 1] - offs[d];
      sorted.append(blob, offs[d], lens[i]);
    }
  }
  std::vector<uint64_t> M;
  if (int rc = gather_rows(c, s, {lens.size(), sorted.size(), (uint64_t)local_err}, &M)) return rc;
  for (int r = 0; r < ws; r++)
    if (M[3 * r + 2]) {
      if (r == me) return set_error(local_err, local_msg.c_str());
      return errf((int)M[3 * r + 2], "rank %d failed in the SHARD name exchange", r);
    }
  uint64_t maxn = 0, maxb = 0;
  for (int r = 0; r < ws; r++) { maxn = std::max(maxn, M[3 * r]); maxb = std::max(maxb, M[3 * r + 1]); }
  std::vector<uint64_t> all_lens((size_t)ws * maxn), mine_l(maxn, 0);
  std::vector<uint8_t> all_bytes((size_t)ws * maxb), mine_b(maxb, 0);
  std::copy(lens.begin(), lens.end(), mine_l.begin());
  std::copy(sorted.begin(), sorted.end(), mine_b.begin());
  if (int rc = coll_gather(c, s, mine_l.data(), all_lens.data(), maxn * 8, false)) return rc;
  if (int rc = coll_gather(c, s, mine_b.data(), all_bytes.data(), maxb, false)) return rc;
  // k-way merge of the sorted lists, distinct names
  struct Cur { uint64_t i = 0, pos = 0; };
  std::vector<Cur> cur(ws);
  c->names.clear();
  c->name_off.assign(1, 0);
  std::vector<uint32_t> my_nid(nd);
  auto name_of = [&](int r, const Cur &x, const uint8_t **p, uint64_t *n) {
    *p = all_bytes.data() + (size_t)r * maxb + x.pos;
    *n = all_lens[(size_t)r * maxn + x.i];
  };
  for (;;) {
    int best = -1;
    const uint8_t *bp = nullptr;
    uint64_t bn = 0;
    for (int r = 0; r < ws; r++) {
      if (cur[r].i >= M[3 * r]) continue;
      const uint8_t *p;
      uint64_t n;
      name_of(r, cur[r], &p, &n);
      if (best < 0 || utf16_compare(p, n, bp, bn) < 0) { best = r; bp = p; bn = n; }
    }
    if (best < 0) break;
    const uint32_t id = (uint32_t)(c->name_off.size() - 1);
    c->names.append(reinterpret_cast<const char *>(bp), bn);
    c->name_off.push_back(c->names.size());
    for (int r = 0; r < ws; r++) {                 // every list's copy of this name (byte-equal: same name)
      if (cur[r].i >= M[3 * r]) continue;
      const uint8_t *p;
      uint64_t n;
      name_of(r, cur[r], &p, &n);
      if (n == bn && memcmp(p, bp, n) == 0) {
        if (r == me) my_nid[perm[cur[r].i]] = id;
        cur[r].pos += n;
        cur[r].i++;
      }
    }
  }
  if (c->name_off.size() - 1 >= 0xFFFFFFFFull) return errf(TFIDF_E_CAPACITY, "more than 2^32 - 1 distinct names");
  DHIP(c->d_name_of_doc.reserve(std::max<uint64_t>(nd, 1) * 4));
  if (nd) DHIP(hipMemcpyAsync(c->d_name_of_doc.p, my_nid.data(), nd * 4, hipMemcpyHostToDevice, s));
  DHIP(hipStreamSynchronize(s));
  c->names_gen = gen;
  c->names_ready = true;
  if (n_names) *n_names = c->name_off.size() - 1;
  return TFIDF_OK;
}

extern "C" int tfidf_dist_shard_search(tfidf_index *ix, tfidf_comm *c, const uint8_t *q, uint64_t q_len,
                                       uint64_t *n_out, uint64_t *n_bytes) {
  if (int rc = check_comm(ix, c)) return rc;
  if (!n_out || (!q && q_len)) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  *n_out = 0;
  if (n_bytes) *n_bytes = 0;
  c->last_name.clear();
  c->last_sum.clear();
  c->last_name_bytes = 0;
  c->last_failed = 0;
  if (int rc = query_status(q, q_len)) return rc;
  DevGuard g(index_device(ix));
  hipStream_t s = index_stream(ix);
  const int ws = c->world;
  uint64_t h = 0, maxn = 0;
  // a rank that cannot serve (stale name table, failed local search) is a
  // failed worker: the others' hits are merged without it (Leader.java:67-69)
  Pinned pin;
  int lrc = local_search_status(pin, ix, c, 0, false);
  if (!lrc) lrc = all_keys(pin, c, q, q_len, 0, &h);            // local doc ids
  if (!lrc && h) {
    if (hipSuccess != c->d_tmp.reserve(h * 8)) lrc = errf(TFIDF_E_OOM, "name records: out of device memory");
    if (!lrc) {
      hipLaunchKernelGGL(k_name_records, dim3(grid_of(h)), dim3(256), 0, s, c->d_keys.as<uint64_t>(), h,
                         c->d_name_of_doc.as<uint32_t>(), c->d_tmp.as<uint64_t>());
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(c->d_keys.p, c->d_tmp.p, h * 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
        lrc = errf(TFIDF_E_HIP, "name records: launch failed");
    }
  }
  const std::string lmsg = lrc ? tfidf_last_error() : "";
  std::vector<uint64_t> ns;
  if (int rc = gather_var(c, s, h, 0, lrc, lmsg, 0, 0, false, &ns, &maxn)) return rc;
  uint64_t n = 0;
  std::vector<uint64_t> base(ws);
  for (int r = 0; r < ws; r++) { base[r] = n; n += ns[r]; }
  if (n == 0) return shard_partial(c, lrc, lmsg);
  if (n >= (1ull << 31)) return errf(TFIDF_E_CAPACITY, "too many hits to merge by name");
  // rank-order (name, score) pairs -> stable sort by name id -> per-name sums in rank order
  DHIP(c->d_srt_k.reserve(n * 16 + 2 * ws * 8));
  DHIP(c->d_srt_v.reserve(n * 16));
  uint32_t *k0 = c->d_srt_k.as<uint32_t>(), *k1 = k0 + n;
  uint64_t *rowinfo = reinterpret_cast<uint64_t *>(c->d_srt_k.as<uint8_t>() + n * 16);
  uint32_t *v0 = c->d_srt_v.as<uint32_t>(), *v1 = v0 + n;
  std::vector<uint64_t> info(2 * ws);
  for (int r = 0; r < ws; r++) { info[r] = ns[r]; info[ws + r] = base[r]; }
  DHIP(hipMemcpyAsync(rowinfo, info.data(), 2 * ws * 8, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_split_records, dim3(grid_of(maxn * ws)), dim3(256), 0, s, c->d_all.as<uint64_t>(), maxn, rowinfo,
                     rowinfo + ws, (uint32_t)ws, k0, v0);
  DHIP(hipGetLastError());
  size_t tmp_bytes = 0, t2 = 0;
  DHIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0, k1, v0, v1, (int)n, 0, 32, s));
  DHIP(c->d_seg.reserve(n * 12 + 16));
  uint32_t *head = c->d_seg.as<uint32_t>(), *pos = head + n, *out_name = pos + n;
  DHIP(hipcub::DeviceScan::ExclusiveSum(nullptr, t2, head, pos, (int)n, s));
  const size_t tcap = (std::max(tmp_bytes, t2) + 255) & ~(size_t)255;
  DHIP(c->d_tmp.reserve(tcap + n * 8));
  double *out_sum = reinterpret_cast<double *>(c->d_tmp.as<uint8_t>() + tcap);
  size_t tb = tcap;
  DHIP(hipcub::DeviceRadixSort::SortPairs(c->d_tmp.p, tb, k0, k1, v0, v1, (int)n, 0, 32, s));
  hipLaunchKernelGGL(k_seg_heads, dim3(grid_of(n)), dim3(256), 0, s, k1, n, head);
  tb = tcap;
  DHIP(hipcub::DeviceScan::ExclusiveSum(c->d_tmp.p, tb, head, pos, (int)n, s));
  hipLaunchKernelGGL(k_seg_sums, dim3(grid_of(n)), dim3(256), 0, s, k1, v1, pos, n, out_name, out_sum);
  DHIP(hipGetLastError());
  uint32_t last[2] = {0, 0};
  DHIP(hipMemcpyAsync(&last[0], pos + n - 1, 4, hipMemcpyDeviceToHost, s));
  DHIP(hipMemcpyAsync(&last[1], head + n - 1, 4, hipMemcpyDeviceToHost, s));
  DHIP(hipStreamSynchronize(s));
  const uint64_t nu = (uint64_t)last[0] + last[1];
  c->last_name.resize(nu);
  c->last_sum.resize(nu);
  DHIP(hipMemcpyAsync(c->last_name.data(), out_name, nu * 4, hipMemcpyDeviceToHost, s));
  DHIP(hipMemcpyAsync(c->last_sum.data(), out_sum, nu * 8, hipMemcpyDeviceToHost, s));
  DHIP(hipStreamSynchronize(s));
  uint64_t nb = 0;
  for (uint32_t id : c->last_name) nb += c->name_off[id + 1] - c->name_off[id];
  c->last_name_bytes = nb;
  *n_out = nu;
  if (n_bytes) *n_bytes = nb;
  return shard_partial(c, lrc, lmsg);
}

extern "C" int tfidf_dist_last_hits(const tfidf_comm *c, uint64_t *doc_ids, float *scores, uint64_t cap,
                                    uint64_t *n_out) {
  if (!c || !n_out) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  return write_hits(const_cast<tfidf_comm *>(c), doc_ids, scores, cap, n_out);
}

extern "C" int tfidf_dist_last_failed(const tfidf_comm *c, uint64_t *rank_mask) {
  if (!c || !rank_mask) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  *rank_mask = c->last_failed;
  return TFIDF_OK;
}

extern "C" int tfidf_dist_last_names(const tfidf_comm *c, uint8_t *buf, uint64_t cap, uint64_t *offsets,
                                     double *scores, uint64_t n_cap, uint64_t *n_out, uint64_t *n_bytes) {
  if (!c || !n_out || !n_bytes) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  const uint64_t n = c->last_name.size();
  *n_out = n;
  *n_bytes = c->last_name_bytes;
  if (n > n_cap || c->last_name_bytes > cap || (n && (!offsets || !scores)) || (c->last_name_bytes && !buf))
    return errf(TFIDF_E_BUFFER, "%llu names of %llu bytes", (unsigned long long)n,
                (unsigned long long)c->last_name_bytes);
  uint64_t p = 0;
  offsets[0] = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint32_t id = c->last_name[i];
    const uint64_t a = c->name_off[id], z = c->name_off[id + 1];
    memcpy(buf + p, c->names.data() + a, z - a);
    p += z - a;
    offsets[i + 1] = p;
    scores[i] = c->last_sum[i];
  }
  return TFIDF_OK;
}

// ---------------------------------------------------------------------------
// process model (1): one process, one shard per GPU

namespace {

// one persistent worker thread per shard: a node call runs the per-rank
// orchestration on every shard at once (the collectives need all ranks in flight)
struct ShardPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done;
  std::function<int(uint32_t)> task;
  uint64_t gen = 0;
  uint32_t pending = 0;
  bool stop = false;
  std::vector<int> rc;
  std::vector<std::string> msg;
  explicit ShardPool(uint32_t n) : rc(n), msg(n) {
    for (uint32_t i = 0; i < n; i++)
      th.emplace_back([this, i] {
        uint64_t seen = 0;
        for (;;) {
          std::function<int(uint32_t)> f;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            f = task;
          }
          const int r = f(i);
          std::string m = r ? tfidf_last_error() : "";
          std::lock_guard<std::mutex> lk(mu);
          rc[i] = r;
          msg[i] = std::move(m);
          if (--pending == 0) done.notify_all();
        }
      });
  }
  ~ShardPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  // runs f(shard) on every shard; the first failure (lowest shard) is the result
  int run(std::function<int(uint32_t)> f) {
    {
      std::lock_guard<std::mutex> lk(mu);
      task = std::move(f);
      pending = (uint32_t)th.size();
      gen++;
    }
    cv.notify_all();
    std::unique_lock<std::mutex> lk(mu);
    done.wait(lk, [&] { return pending == 0; });
    for (size_t i = 0; i < rc.size(); i++)
      if (rc[i]) return set_error(rc[i], ("shard " + std::to_string(i) + ": " + msg[i]).c_str());
    return TFIDF_OK;
  }
};

}  // namespace

struct tfidf_node {
  tfidf_config cfg;
  std::vector<int> devices;
  std::vector<tfidf_index *> shards;
  std::vector<tfidf_comm *> comms;
  std::vector<uint64_t> doc_base;
  std::unique_ptr<ShardPool> pool;
  std::mutex mu;                     // node calls are serialised
  int transport = TFIDF_TRANSPORT_INPROC;
  bool committed = false;
  uint64_t num_docs = 0, doc_count = 0, sum_ttf = 0, num_terms = 0;
};

extern "C" int tfidf_node_create_devices(const tfidf_config *cfg, const int32_t *devices, uint32_t n_devices,
                                         uint32_t flags, tfidf_node **out) {
  if (!cfg || !devices || !out || n_devices == 0) return errf(TFIDF_E_INVALID_ARG, "NULL argument or no devices");
  if (n_devices > 64) return errf(TFIDF_E_INVALID_ARG, "at most 64 shards");
  std::unique_ptr<tfidf_node> n(new tfidf_node());
  n->cfg = *cfg;
  bool repeat = false;
  for (uint32_t i = 0; i < n_devices; i++) {
    for (uint32_t j = 0; j < i; j++) repeat |= devices[j] == devices[i];
    n->devices.push_back(devices[i]);
  }
  const bool inproc = repeat || (flags & TFIDF_NODE_INPROC);
  for (uint32_t i = 0; i < n_devices; i++) {
    tfidf_config c = *cfg;
    c.device = devices[i];
    tfidf_index *ix = nullptr;
    if (int rc = tfidf_create(&c, &ix)) {
      for (tfidf_index *x : n->shards) tfidf_destroy(x);
      return rc;
    }
    n->shards.push_back(ix);
  }
  if (inproc) {
    n->comms.resize(n_devices);
    tfidf_comm_create_inproc((int32_t)n_devices, n->comms.data());
    for (uint32_t i = 0; i < n_devices; i++) n->comms[i]->device = devices[i];
    n->transport = TFIDF_TRANSPORT_INPROC;
  } else {
    RcclApi &api = rccl();
    int rc = api.ok ? TFIDF_OK : errf(TFIDF_E_NO_DEVICE, "%s", api.err.c_str());
    std::vector<ncclComm_t> cm(n_devices, nullptr);
    if (!rc) {
      ncclResult_t r = api.CommInitAll(cm.data(), (int)n_devices, devices);
      if (r != ncclSuccess) rc = errf(TFIDF_E_HIP, "ncclCommInitAll: %s", api.GetErrorString(r));
    }
    if (rc) {
      for (tfidf_index *x : n->shards) tfidf_destroy(x);
      return rc;
    }
    for (uint32_t i = 0; i < n_devices; i++) {
      tfidf_comm *c = new tfidf_comm();
      c->rank = (int)i;
      c->world = (int)n_devices;
      c->device = devices[i];
      c->t.reset(new RcclTransport(cm[i], (int)n_devices));
      n->comms.push_back(c);
    }
    n->transport = TFIDF_TRANSPORT_RCCL;
  }
  n->doc_base.assign(n_devices, 0);
  n->pool.reset(new ShardPool(n_devices));
  *out = n.release();
  return TFIDF_OK;
}

extern "C" int tfidf_node_create(const tfidf_config *cfg, uint64_t device_mask, tfidf_node **out) {
  std::vector<int32_t> dev;
  for (int i = 0; i < 64; i++)
    if ((device_mask >> i) & 1u) dev.push_back(i);
  if (dev.empty()) return errf(TFIDF_E_INVALID_ARG, "empty device mask");
  return tfidf_node_create_devices(cfg, dev.data(), (uint32_t)dev.size(), 0, out);
}

extern "C" int tfidf_node_destroy(tfidf_node *n) {
  if (!n) return TFIDF_OK;
  n->pool.reset();
  for (tfidf_comm *c : n->comms) {
    DevGuard g(n->devices[c->rank]);
    delete c;
  }
  for (tfidf_index *x : n->shards) tfidf_destroy(x);
  delete n;
  return TFIDF_OK;
}

extern "C" int tfidf_node_shard(tfidf_node *n, uint32_t i, tfidf_index **ix, uint32_t *n_shards) {
  if (!n) return errf(TFIDF_E_INVALID_ARG, "NULL node");
  if (n_shards) *n_shards = (uint32_t)n->shards.size();
  if (ix) {
    if (i >= n->shards.size()) return errf(TFIDF_E_INVALID_ARG, "shard %u out of range", i);
    *ix = n->shards[i];
  }
  return TFIDF_OK;
}

extern "C" int tfidf_node_add_docs(tfidf_node *n, int32_t shard, const uint8_t *utf8, const uint64_t *offsets,
                                   uint64_t n_docs, const uint8_t *keys, const uint64_t *key_offsets) {
  if (!n || !offsets) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(n->mu);
  const uint32_t G = (uint32_t)n->shards.size();
  if (shard >= (int32_t)G || shard < -1) return errf(TFIDF_E_INVALID_ARG, "shard %d out of range", shard);
  n->committed = false;
  if (shard >= 0) return tfidf_add_docs(n->shards[shard], utf8, offsets, n_docs, keys, key_offsets);
  // contiguous split: shard g takes documents [g N / G, (g + 1) N / G)
  return n->pool->run([&](uint32_t g) {
    const uint64_t lo = g * n_docs / G, hi = (g + 1) * n_docs / G;
    return tfidf_add_docs(n->shards[g], utf8, offsets + lo, hi - lo, keys, keys ? key_offsets + lo : nullptr);
  });
}

extern "C" int tfidf_node_commit(tfidf_node *n) {
  if (!n) return errf(TFIDF_E_INVALID_ARG, "NULL node");
  std::lock_guard<std::mutex> lk(n->mu);
  n->committed = false;
  // 1. every shard's own commit (all of them, before any collective: a shard
  //    that fails must not leave the others waiting in an exchange)
  if (int rc = n->pool->run([&](uint32_t g) { return tfidf_commit(n->shards[g]); })) return rc;
  uint64_t base = 0, dc = 0, ttf = 0;
  for (size_t g = 0; g < n->shards.size(); g++) {
    tfidf_index_stats st{};
    if (int rc = tfidf_stats(n->shards[g], &st)) return rc;
    n->doc_base[g] = base;
    base += st.num_docs;
    dc += st.doc_count;
    ttf += st.sum_ttf;
  }
  if (base > (1ull << 32)) return errf(TFIDF_E_CAPACITY, "more than 2^32 documents on the node");
  n->num_docs = base;
  // 2. GLOBAL statistics, or the SHARD name table
  if (n->cfg.stats_mode == TFIDF_STATS_GLOBAL) {
    std::vector<uint64_t> nv(n->shards.size()), gdc(n->shards.size()), gttf(n->shards.size());
    if (int rc = n->pool->run([&](uint32_t g) {
          return tfidf_dist_global_commit(n->shards[g], n->comms[g], &nv[g], &gdc[g], &gttf[g]);
        }))
      return rc;
    n->num_terms = nv[0];
    n->doc_count = gdc[0];
    n->sum_ttf = gttf[0];
  } else {
    if (int rc = n->pool->run([&](uint32_t g) { return tfidf_dist_shard_commit(n->shards[g], n->comms[g], nullptr); }))
      return rc;
    n->num_terms = 0;
    n->doc_count = dc;
    n->sum_ttf = ttf;
  }
  n->committed = true;
  return TFIDF_OK;
}

extern "C" int tfidf_node_search(tfidf_node *n, const uint8_t *q, uint64_t q_len, uint32_t k, uint64_t *doc_ids,
                                 float *scores, uint64_t cap, uint64_t *n_out) {
  if (!n || !n_out) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(n->mu);
  *n_out = 0;
  if (!n->committed) return errf(TFIDF_E_STATE, "search before tfidf_node_commit");
  if (n->cfg.stats_mode != TFIDF_STATS_GLOBAL) return errf(TFIDF_E_STATE, "GLOBAL mode only (tfidf_node_search_names)");
  if (int rc = n->pool->run([&](uint32_t g) {
        uint64_t m = 0;
        const int r = tfidf_dist_search(n->shards[g], n->comms[g], n->doc_base[g], q, q_len, k, nullptr, nullptr, 0, &m);
        return r == TFIDF_E_BUFFER ? TFIDF_OK : r;
      }))
    return rc;
  return write_hits(n->comms[0], doc_ids, scores, cap, n_out);
}

extern "C" int tfidf_node_search_batch(tfidf_node *n, const uint8_t *q_utf8, const uint64_t *q_offsets, uint32_t n_q,
                                       uint32_t k, uint64_t *doc_ids, float *scores, uint32_t *counts) {
  if (!n) return errf(TFIDF_E_INVALID_ARG, "NULL node");
  std::lock_guard<std::mutex> lk(n->mu);
  if (!n->committed) return errf(TFIDF_E_STATE, "search before tfidf_node_commit");
  if (n->cfg.stats_mode != TFIDF_STATS_GLOBAL) return errf(TFIDF_E_STATE, "GLOBAL mode only");
  if (k == 0 || k > 1024) return errf(TFIDF_E_INVALID_ARG, "1 <= k <= 1024");
  const size_t per = (size_t)n_q * k;
  std::vector<std::vector<uint64_t>> d(n->shards.size());
  std::vector<std::vector<float>> sc(n->shards.size());
  std::vector<std::vector<uint32_t>> ct(n->shards.size());
  // shard 0 writes the caller's arrays; the others' (identical) copies are scratch
  return n->pool->run([&](uint32_t g) {
    uint64_t *pd = doc_ids;
    float *ps = scores;
    uint32_t *pc = counts;
    if (g) {
      d[g].resize(per);
      sc[g].resize(per);
      ct[g].resize(n_q);
      pd = d[g].data();
      ps = sc[g].data();
      pc = ct[g].data();
    }
    return tfidf_dist_search_batch(n->shards[g], n->comms[g], n->doc_base[g], q_utf8, q_offsets, n_q, k, pd, ps, pc);
  });
}

extern "C" int tfidf_node_search_names(tfidf_node *n, const uint8_t *q, uint64_t q_len, uint8_t *buf, uint64_t cap,
                                       uint64_t *offsets, double *scores, uint64_t n_cap, uint64_t *n_out,
                                       uint64_t *n_bytes) {
  if (!n || !n_out || !n_bytes) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(n->mu);
  *n_out = *n_bytes = 0;
  if (!n->committed) return errf(TFIDF_E_STATE, "search before tfidf_node_commit");
  if (n->cfg.stats_mode != TFIDF_STATS_SHARD) return errf(TFIDF_E_STATE, "SHARD mode only (tfidf_node_search)");
  std::vector<std::string> why(n->shards.size());
  if (int rc = n->pool->run([&](uint32_t g) {
        uint64_t m = 0, b = 0;
        const int r = tfidf_dist_shard_search(n->shards[g], n->comms[g], q, q_len, &m, &b);
        if (r == TFIDF_OK && n->comms[g]->last_failed) why[g] = tfidf_last_error();
        return r;
      }))
    return rc;
  const int rc = tfidf_dist_last_names(n->comms[0], buf, cap, offsets, scores, n_cap, n_out, n_bytes);
  if (rc == TFIDF_OK && n->comms[0]->last_failed) {        // partial answer: say which shards were skipped
    std::string m = why[0];
    for (size_t g = 0; g < why.size(); g++)
      if ((n->comms[0]->last_failed >> g) & 1u) m += "; shard " + std::to_string(g) + ": " + why[g];
    set_error(TFIDF_OK, m.c_str());
  }
  return rc;
}

extern "C" int tfidf_node_last_failed(const tfidf_node *n, uint64_t *shard_mask) {
  if (!n || !shard_mask) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  *shard_mask = n->comms.empty() ? 0 : n->comms[0]->last_failed;
  return TFIDF_OK;
}

extern "C" int tfidf_node_doc_key(tfidf_node *n, uint64_t doc, uint8_t *buf, uint64_t cap, uint64_t *n_out) {
  if (!n || !n_out) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  std::lock_guard<std::mutex> lk(n->mu);
  if (!n->committed) return errf(TFIDF_E_STATE, "not committed");
  if (doc >= n->num_docs) return errf(TFIDF_E_INVALID_ARG, "doc out of range");
  size_t g = n->shards.size() - 1;
  while (n->doc_base[g] > doc) g--;
  return tfidf_doc_key(n->shards[g], doc - n->doc_base[g], buf, cap, n_out);
}

extern "C" int tfidf_node_stats_get(const tfidf_node *n, tfidf_node_stats *out) {
  if (!n || !out) return errf(TFIDF_E_INVALID_ARG, "NULL argument");
  out->n_shards = n->shards.size();
  out->num_docs = n->num_docs;
  out->doc_count = n->doc_count;
  out->sum_ttf = n->sum_ttf;
  out->num_terms = n->num_terms;
  out->transport = (uint64_t)n->transport;
  return TFIDF_OK;
}
