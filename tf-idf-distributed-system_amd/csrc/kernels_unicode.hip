// kernels_unicode.hip — index build of documents holding non-ASCII text
// (Worker.addDocToIndex, Worker.java:190-220, through StandardAnalyzer's full
// Unicode grammar; unicode_scan.h), hand-written for gfx950.
//
//   tokenize_uwave : one wavefront per document (aligned window <= 4 KB), the
//                    documents the ASCII wave path flagged (a byte >= 0x80).
//                    The document is staged in LDS with per-byte classes;
//                    lane l scans the slice [cut_l, cut_{l+1}) with the
//                    longest-match DFA, cuts just after ASCII class-OTHER
//                    bytes (the scanner's start state holds there); every
//                    round each lane yields at most one token, keyed
//                    (lower-cased UTF-8 -> 128-bit key; <= 8 ASCII bytes
//                    directly), and the wave inserts the round's keys into a
//                    512-slot LDS table (64-bit CAS on lo, then hi; in-order
//                    LDS within the wave makes the winner's hi visible to the
//                    losers of the same round).  The occupied slots are
//                    compacted, resolved in the global dictionary (4 lookups
//                    per lane in flight) and written as a CSR row grouped by
//                    dictionary range, as the other tokenizer paths do.
//                    Documents that do not fit (window, > 512 distinct terms,
//                    malformed UTF-8) go to the long path.
//   tokenize_uchunk: the same scanner over the (document, 2 KB core) units of
//                    book-sized documents whose window holds non-ASCII text.
#include <hip/hip_runtime.h>

#include "dict_device.h"
#include "tfidf_common.h"
#include "tfidf_internal.h"
#include "unicode_scan.h"

namespace tfidf {

constexpr uint32_t kUwWindow = 4096;
constexpr uint32_t kUwSlots = 512;
constexpr uint32_t kUwSlotBits = 9;
constexpr uint32_t kUwMaxTerms = 512;
constexpr uint32_t kUwMaxRanges = 64;

// Scanner class source over classes precomputed in LDS: per byte, the class
// of the char starting there | (length - 1) << 5, or 0xFF (malformed, or a
// continuation byte: a scan never lands on one of a well-formed char).
struct UwClassSrcRef {
  const uint8_t *cls;
  __device__ __forceinline__ uint32_t at(uint64_t i, uint32_t *len) const {
    const uint32_t v = cls[i];
    if (v == 0xFFu) return kUcBad;
    *len = (v >> 5) + 1;
    return v & 31u;
  }
};

constexpr uint32_t kUwClasses = 19;     // kUc* classes
constexpr uint32_t kUwStates = 12;      // kW* states (incl. kWDead)

// WORD-rule scan over chars (not units), from *pos up to stop: the next token
// span [*ts, *te).  An extender keeps the DFA state (it belongs to the unit
// of the preceding head), any other class takes a transition of the LDS table
// built from uc_word_next; the same spans as uc_next_span (unicode_scan.h),
// with one LDS read per char for the class and one for the transition.  Runs
// of ASCII letters / digits are skipped four class bytes per LDS read.
// *at_end = the scan reached byte n while a longer match was still possible
// (a window that ends there, not the document: the token's extent is unknown)
__device__ __forceinline__ bool uc_window_span(const uint8_t *cls, const uint8_t *tr, uint32_t n, uint32_t *pos,
                                               uint32_t stop, uint32_t *ts, uint32_t *te, bool *bad, bool *at_end) {
  while (*pos < stop) {
    const uint32_t i = *pos;
    const uint32_t v = cls[i];
    if (v == 0xFFu) { *bad = true; return false; }
    const uint32_t c = v & 31u, l = (v >> 5) + 1;
    const uint32_t st0 = tr[kWStart * kUwClasses + c];
    if (st0 != kWDead) {
      uint32_t st = st0, p = i + l, last = uc_word_accepting(st) ? p : i, erun = p;
      bool dead = false;
      while (p < n) {
        if (st == kWA || st == kWN) {
          // ASCII letters / digits (class bytes 0x01 / 0x03) keep the state in
          // {A, N} (WB5, WB8-WB10), both accepting: skip the run four class
          // bytes per aligned LDS read instead of a DFA step per byte
          const uint32_t *c32 = reinterpret_cast<const uint32_t *>(cls);
          uint32_t q = p;
          while (q < n) {
            const uint32_t x = __builtin_amdgcn_alignbyte(c32[(q >> 2) + 1], c32[q >> 2], q & 3);
            const uint32_t m = (x & 0xFDFDFDFDu) ^ 0x01010101u;          // zero byte: ASCII alnum
            const uint32_t run = m ? (uint32_t)__builtin_ctz(m) >> 3 : 4u;
            q += min(run, n - q);
            if (run < 4) break;
          }
          if (q > p) {
            st = cls[q - 1] == 0x01u ? kWA : kWN;
            p = q;
            last = p;
            if (p >= n) break;
          }
        }
        const uint32_t w = cls[p];
        if (w == 0xFFu) { *bad = true; return false; }
        const uint32_t cw = w & 31u;
        if (!uc_is_extender(cw)) {
          const uint32_t ns = tr[st * kUwClasses + cw];
          if (ns == kWDead) { dead = true; break; }
          st = ns;
        }
        p += (w >> 5) + 1;
        if (uc_word_accepting(st)) last = p;
        else if (st == kWELead) erun = p;
      }
      if (!dead) *at_end = true;
      if (last > i) { *ts = i; *te = last; *pos = last; return true; }
      uint32_t q = i + l;
      while (q < erun && (cls[q] & 31u) != kUcExtendSA) q += (cls[q] >> 5) + 1;
      *pos = q;
      continue;
    }
    if (c == kUcOther || c == kUcExtend || c == kUcZWJ || c == kUcMidLetter || c == kUcMidNumLet ||
        c == kUcMidNum || c == kUcSQuote || c == kUcDQuote) {
      *pos = i + l;
      continue;
    }
    const UwClassSrcRef src{cls};
    uint64_t p64 = i, ts64, te64;
    if (!uc_next_span(src, n, &p64, (uint64_t)i + 1, &ts64, &te64, bad)) {
      *pos = (uint32_t)p64;
      if (*bad) return false;
      continue;
    }
    // SA runs / Han / emoji units: conservatively, a span ending near the window end is unknown
    if (te64 + 8 >= n) *at_end = true;
    *ts = (uint32_t)ts64; *te = (uint32_t)te64; *pos = (uint32_t)p64;
    return true;
  }
  return false;
}

// Key of a token of n <= 8 bytes at (aligned) window byte a when they are all
// ASCII: the lower-cased bytes, as KeyBuilder gives them (uc_token_key's
// UTF-8 walk is for the rest).  false: a byte >= 0x80.
__device__ __forceinline__ uint32_t uc_lower4(uint32_t t) {
  const uint32_t up = (t + 0x3F3F3F3Fu) & ~(t + 0x25252525u) & 0x80808080u;   // 'A'..'Z' (ASCII bytes)
  return t | (up >> 2);
}
__device__ __forceinline__ bool uc_short_ascii_key(const uint8_t *text, uint32_t a, uint32_t n, uint64_t *lo) {
  const uint32_t *t32 = reinterpret_cast<const uint32_t *>(text);
  const uint32_t w0 = t32[a >> 2], w1 = t32[(a >> 2) + 1], w2 = t32[(a >> 2) + 2], o = a & 3;
  uint32_t x0 = __builtin_amdgcn_alignbyte(w1, w0, o), x1 = __builtin_amdgcn_alignbyte(w2, w1, o);
  x0 &= n >= 4 ? 0xFFFFFFFFu : (1u << (8 * n)) - 1u;
  x1 &= n >= 8 ? 0xFFFFFFFFu : (n <= 4 ? 0u : (1u << (8 * (n - 4))) - 1u);
  if ((x0 | x1) & 0x80808080u) return false;
  *lo = (uint64_t)uc_lower4(x0) | ((uint64_t)uc_lower4(x1) << 32);
  return true;
}

struct UwSmem {
  alignas(16) uint8_t text[kUwWindow + 16];
  alignas(16) uint8_t cls[kUwWindow + 16];
  unsigned long long klo[kUwSlots];   // key lo; after the lookup: dictionary slot
  unsigned long long khi[kUwSlots];   // key hi (VALID bit set: occupied)
  uint32_t cnt[kUwSlots];             // tf
  uint32_t kpos[kUwSlots];            // first occurrence: start | end << 16 (document bytes)
  uint16_t occ[kUwSlots];             // occupied slots, compacted
  uint32_t rcnt[kUwMaxRanges];        // per-range counts, then cursors
  uint8_t tr[kUwStates * kUwClasses]; // WORD DFA transitions
  uint8_t asc[128];                   // ASCII byte -> scanner class
  uint32_t isl[64];                   // sparse path: islands (window start | end << 16)
  uint32_t n_isl, n_tok;              // sparse path: counters
};

__device__ __forceinline__ uint32_t uw_incl_add(uint32_t x, uint32_t lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  return x;
}


// ---------------------------------------------------------------------------
// Sparse non-ASCII documents (round 5): most of a real document is ASCII
// words with a few non-ASCII chars (accents, curly quotes).  A token never
// crosses an ASCII byte of class OTHER (a split byte) and JFlex never looks
// behind, so the document splits into pieces between split bytes that scan
// independently from the start state.  Pieces without a byte >= 0x80 take the
// ASCII word rules of the wave tokenizer (SWAR word masks, token spans by bit
// operations: the same tokens as the scanner there); only the "islands" —
// pieces holding a non-ASCII byte — go through the longest-match scanner, one
// island per lane.  Every token lands in a dense list, inserted into the
// document's table 64 per round (no lane waits on another lane's scan).
// Documents whose non-ASCII text is not sparse (more than kUwIslands islands,
// a piece over kUwMaxPiece bytes, more island bytes than the class buffer, an
// ASCII token over 255 chars, more than kUwTokens tokens, malformed UTF-8)
// take the full per-lane scan below.
constexpr uint32_t kUwTokens = 1024;       // token list (in the class-byte area)
constexpr uint32_t kUwIslands = 64;
constexpr uint32_t kUwIslandBytes = kUwSlots * 2 - 32;   // island class bytes (in the occ area, + read slack)
constexpr uint32_t kUwMaxPiece = 512;
static_assert(kUwTokens * 4 <= kUwWindow, "token list in cls");

__device__ __forceinline__ uint32_t uw_eq(uint32_t x, uint32_t c4) { return ~((x ^ c4) + 0x7F7F7F7Fu) & 0x80808080u; }
__device__ __forceinline__ uint32_t uw_letter(uint32_t x) {
  const uint32_t lw = x | 0x20202020u;
  return (lw + 0x1F1F1F1Fu) & ~(lw + 0x05050505u) & 0x80808080u;
}
__device__ __forceinline__ uint32_t uw_digit(uint32_t x) { return (x + 0x50505050u) & ~(x + 0x46464646u) & 0x80808080u; }
__device__ __forceinline__ uint32_t uw_nib(uint32_t w) {
  const uint32_t f = (w >> 7) & 0x01010101u;
  const uint32_t g = f | (f >> 7);
  return (g | (g >> 14)) & 0xFu;
}
__device__ __forceinline__ uint32_t uw_keep(uint32_t q, uint32_t lo, uint32_t hi) {   // bytes of dword q in [lo, hi)
  const uint32_t a = q >= lo ? 0xFFFFFFFFu : (lo - q >= 4 ? 0u : (0xFFFFFFFFu << (8 * (lo - q))));
  const uint32_t b = q + 4 <= hi ? 0xFFFFFFFFu : (hi <= q ? 0u : (0xFFFFFFFFu >> (8 * (q + 4 - hi))));
  return a & b;
}
__device__ __forceinline__ bool uw_split_at(const uint8_t *text, uint32_t w, uint32_t lo, uint32_t hi) {
  return w < lo || w >= hi || uc_split_byte(text[w]);
}

// Masks of window bytes [64 lane, 64 lane + 64), document bytes [lo, hi):
// *W ASCII word bytes (letters, digits, '_', joiners between letters / digits:
// the wave tokenizer's rules), *NA bytes >= 0x80, *SP split bytes (ASCII class
// OTHER, and every byte outside the document).  Non-ASCII bytes are cleared
// before the byte-wise arithmetic (no carries) and are never word bytes here.
__device__ __forceinline__ void uw_lane_masks(const uint8_t *text, uint32_t lane, uint32_t lo, uint32_t hi,
                                              uint64_t *W, uint64_t *NA, uint64_t *SP) {
  uint32_t x[16];
  {
    const uint4 *t = reinterpret_cast<const uint4 *>(text + lane * 64);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 v = t[k];
      x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
    }
  }
  uint32_t LD[16];
  uint64_t na = 0, sp = 0;
  bool mid = false;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    x[i] &= uw_keep(64 * lane + 4 * i, lo, hi);
    const uint32_t hb = x[i] & 0x80808080u;
    na |= (uint64_t)uw_nib(hb) << (4 * i);
    x[i] &= ~((hb >> 7) * 0xFFu);
    const uint32_t D = uw_digit(x[i]), Lt = uw_letter(x[i]);
    LD[i] = Lt | (D >> 1);
    const uint32_t j = uw_eq(x[i], 0x3A3A3A3Au) | uw_eq(x[i], 0x2E2E2E2Eu) | uw_eq(x[i], 0x2C2C2C2Cu) |
                       uw_eq(x[i], 0x3B3B3B3Bu) | uw_eq(x[i], 0x27272727u);
    mid |= j != 0;
    const uint32_t keep = Lt | D | j | uw_eq(x[i], 0x5F5F5F5Fu) | uw_eq(x[i], 0x22222222u);
    sp |= (uint64_t)uw_nib(~keep & 0x80808080u) << (4 * i);
  }
  uint32_t ldp = (uint32_t)__shfl_up((int)LD[15], 1, 64);
  uint32_t ldn = (uint32_t)__shfl_down((int)LD[0], 1, 64);
  if (lane == 0) ldp = 0;
  if (lane == 63) ldn = 0;
  const bool mids = __any(mid);
  uint64_t w = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t c = LD[i] | (LD[i] << 1) | uw_eq(x[i], 0x5F5F5F5Fu);
    if (mids) {
      const uint32_t prev4 = i ? LD[i - 1] : ldp;
      const uint32_t next4 = i < 15 ? LD[i + 1] : ldn;
      const uint32_t pf = __builtin_amdgcn_alignbyte(LD[i], prev4, 3);
      const uint32_t nf = __builtin_amdgcn_alignbyte(next4, LD[i], 1);
      const uint32_t both = pf & nf;
      const uint32_t dq = uw_eq(x[i], 0x2E2E2E2Eu) | uw_eq(x[i], 0x27272727u);
      const uint32_t ml = dq | uw_eq(x[i], 0x3A3A3A3Au);
      const uint32_t mn = dq | uw_eq(x[i], 0x2C2C2C2Cu) | uw_eq(x[i], 0x3B3B3B3Bu);
      c |= (ml & both) | (mn & (both << 1));
    }
    w |= (uint64_t)uw_nib(c & 0x80808080u) << (4 * i);
  }
  *W = w;
  *NA = na;
  *SP = sp & ~na;
}

// The sparse path's token list: sm.cls as u32 entries (document start | end
// << 16).  Returns false (wave-uniform) when the document must take the full
// scan; else *ntok entries are listed.
__device__ __forceinline__ bool uw_sparse_tokens(UwSmem &sm, const BuildParams &p, uint32_t lane, uint32_t shift, uint32_t L,
                                 uint32_t *ntok) {
  const uint32_t lo = shift, hi = shift + L;
  uint64_t W, NA, SP;
  uw_lane_masks(sm.text, lane, lo, hi, &W, &NA, &SP);
  if (lane == 0) { sm.n_isl = 0; sm.n_tok = 0; }
  __syncthreads();
  // islands: the first non-ASCII byte of each piece finds the piece's ends
  bool fb = false;
  {
    uint64_t m = NA;
    uint32_t prev = 0xFFFFFFFFu;                        // previous non-ASCII bit of this lane
    while (m) {
      const uint32_t b = (uint32_t)__builtin_ctzll(m);
      m &= m - 1;
      // a non-ASCII byte of this lane before it with no split byte in between: same piece
      if (prev != 0xFFFFFFFFu && ((SP >> prev) & ((1ull << (b - prev)) - 1)) == 0) { prev = b; continue; }
      prev = b;
      const uint32_t w = 64 * lane + b;
      uint32_t a = w;                                   // piece start: after the last split byte
      bool first = true;
      while (!uw_split_at(sm.text, a - 1, lo, hi)) {
        if (sm.text[a - 1] >= 0x80u) { first = false; break; }
        if (w - a >= kUwMaxPiece) { fb = true; break; }
        a--;
      }
      if (!first || fb) continue;
      uint32_t z = w + 1;                               // piece end: the next split byte
      while (!uw_split_at(sm.text, z, lo, hi)) {
        if (z - a >= kUwMaxPiece) { fb = true; break; }
        z++;
      }
      if (fb) continue;
      const uint32_t at = atomicAdd(&sm.n_isl, 1u);
      if (at < kUwIslands) sm.isl[at] = a | (z << 16);
      else fb = true;
    }
  }
  __syncthreads();
  const uint32_t n_isl = sm.n_isl;
  if (__any(fb) || n_isl > kUwIslands) return false;
  // ASCII tokens outside the islands
  {
    const uint32_t w0 = 64 * lane;
    uint64_t I = 0;
    for (uint32_t j = 0; j < n_isl; j++) {
      const uint32_t e = sm.isl[j], a = max(e & 0xFFFFu, w0), z = min(e >> 16, w0 + 64);
      if (a < z) I |= (z - a == 64 ? ~0ull : ((1ull << (z - a)) - 1)) << (a - w0);
    }
    W &= ~I;
  }
  const uint64_t wlast = __ballot((W >> 63) & 1ull);
  const uint64_t prevW = lane ? (wlast >> (lane - 1)) & 1ull : 0ull;
  const uint64_t S = W & ~((W << 1) | prevW);
  uint64_t E = ~W & ((W << 1) | prevW);
  const uint32_t firstE = E ? lane * 64 + (uint32_t)__builtin_ctzll(E) : kUwWindow;
  const uint64_t hasE = __ballot(E != 0);
  const uint64_t later = lane == 63 ? 0ull : (hasE & (~0ull << (lane + 1)));
  const uint32_t srcl = later ? (uint32_t)__builtin_ctzll(later) : lane;
  uint32_t nz = (uint32_t)__shfl((int)firstE, (int)srcl, 64);
  if (!later) nz = kUwWindow;
  if (prevW) E &= E - 1;                                // closes the token open from lane - 1
  const uint32_t nts = (uint32_t)__popcll(S);
  const uint32_t incl = uw_incl_add(nts, lane);
  const uint32_t nasc = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (nasc > kUwTokens) return false;
  uint32_t *tok = reinterpret_cast<uint32_t *>(sm.cls);
  bool toolong = false;
  {
    uint32_t at = incl - nts;
    uint64_t s = S, e = E;
    while (s) {
      const uint32_t tp = lane * 64 + (uint32_t)__builtin_ctzll(s);
      const uint32_t te = e ? lane * 64 + (uint32_t)__builtin_ctzll(e) : nz;
      s &= s - 1;
      e &= e - 1;
      toolong |= te - tp > kMaxTokenLen;
      tok[at++] = (tp - shift) | ((te - shift) << 16);
    }
  }
  if (__any(toolong)) return false;                     // the 255-char cut: the full scan does it
  if (lane == 0) sm.n_tok = nasc;
  // island class bytes (in the occ area): island j at an offset congruent to
  // its document start mod 4, so the scanner's aligned 4-byte class reads line up
  uint8_t *cb = reinterpret_cast<uint8_t *>(sm.occ);
  uint32_t a = 0, z = 0;
  const bool mine = lane < n_isl;
  if (mine) {
    const uint32_t e = sm.isl[lane];
    a = (e & 0xFFFFu) - shift;
    z = (e >> 16) - shift;
  }
  const uint32_t need = mine ? ((z - a + 1 + 3) & ~3u) + 8 : 0u;
  const uint32_t ni = uw_incl_add(need, lane);
  if ((uint32_t)__builtin_amdgcn_readlane((int)ni, 63) > kUwIslandBytes) return false;
  const uint32_t off = ni - need + (a & 3);
  bool bad = false;
  if (mine) {
    const uint8_t *doc = sm.text + shift;
    const uint32_t zc = min(z + 1, L);                  // the split byte at z closes the scan
    for (uint32_t i = a; i < zc; i++) {
      const uint32_t x = doc[i];
      uint32_t v;
      if (x < 0x80u) v = sm.asc[x];
      else if ((x & 0xC0u) == 0x80u) v = 0xFFu;
      else {
        uint32_t l;
        const uint32_t cp = utf8_decode(doc, L, i, &l);
        v = cp == kUcBad ? 0xFFu : (uc_class(cp) | ((l - 1) << 5));
      }
      cb[off + (i - a)] = (uint8_t)v;
    }
  }
  __syncthreads();
  if (mine) {
    const uint8_t *cl = cb + off - a;                   // class byte of document position i: cl[i]
    const uint32_t n = min(z + 1, L);
    uint32_t pos = a, ts, te;
    bool at_end = false;
    while (pos < z && uc_window_span(cl, sm.tr, n, &pos, z, &ts, &te, &bad, &at_end)) {
      if (te - ts > kMaxTokenLen) {                     // > 255 bytes: maybe > 255 UTF-16 units (cut)
        uint64_t klo, khi;
        const uint64_t cut = uc_token_key(sm.text + shift, L, ts, te, &klo, &khi, p.hash_seed);
        if (cut < te) { te = (uint32_t)cut; pos = te; }
      }
      const uint32_t at = atomicAdd(&sm.n_tok, 1u);
      if (at < kUwTokens) tok[at] = ts | (te << 16);
    }
  }
  __syncthreads();
  *ntok = sm.n_tok;
  return !__any(bad) && *ntok <= kUwTokens;
}

// Documents flagged by k_tokenize_wave (uni_list[d] != 0: a flag per
// document, no shared counter — a list appended with one atomic per document
// serialised a corpus of non-ASCII documents on one address, ~4.7 ns each):
// the wave reads 64 flags at a time, takes the flagged documents of each
// group in turn and counts them into *uni_count.  Round 4: classes four
// consecutive bytes per lane (no LDS bank conflicts), the ASCII-run skip and
// the direct key of short ASCII tokens of the Unicode chunk kernel,
// dictionary lookups and row writes over the compacted occupied slots only
// (was: all 1 024 slots, two rounds), occupied slots reset after the document
// instead of a full table clear.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_tokenize_uwave(BuildParams p) {
  __shared__ UwSmem sm;
  const uint32_t lane = threadIdx.x;
  const uint32_t R = p.n_ranges;
  unsigned long long my_dc = 0, my_ttf = 0, my_nnz = 0;
  uint32_t my_uni = 0;
  bool ready = false;                                       // tables built (at the first flagged document)

  for (uint64_t b0 = (uint64_t)blockIdx.x * 64; b0 < p.n_docs; b0 += (uint64_t)gridDim.x * 64) {
    uint64_t fm = __ballot(b0 + lane < p.n_docs && p.uni_list[b0 + lane] != 0);
    my_uni += (uint32_t)__popcll(fm);
    while (fm) {
    const uint32_t d = (uint32_t)(b0 + (uint64_t)__builtin_ctzll(fm));
    fm &= fm - 1;
    if (!ready) {                                           // wave-uniform
      for (uint32_t e = lane; e < kUwStates * kUwClasses; e += 64)
        sm.tr[e] = (uint8_t)uc_word_next(e / kUwClasses, e % kUwClasses);
      for (uint32_t e = lane; e < 128; e += 64) sm.asc[e] = (uint8_t)uc_ascii_class(e);
      for (uint32_t s = lane; s < kUwSlots; s += 64) { sm.klo[s] = 0; sm.khi[s] = 0; sm.cnt[s] = 0; }
      __syncthreads();
      ready = true;
    }
    const uint64_t src = p.live_map ? p.live_map[d] : d;
    const uint64_t s0 = p.offsets[src];
    const uint64_t L = p.offsets[src + 1] - s0;
    if (L > kUwWindow || R > kUwMaxRanges) {                // wave-uniform
      if (lane == 0) p.long_list[atomicAdd(p.long_count, 1u)] = d;
      if (L > kUwWindow) my_uni--;                          // (UNI-first builds flag long documents too: a long
                                                            // document is not counted as non-ASCII, as the ASCII pass has it)
      continue;
    }
    // ---- stage (aligned 16 B loads); the table is empty here
    const uintptr_t a = reinterpret_cast<uintptr_t>(p.text + s0);
    const uint32_t shift = (uint32_t)(a & 15);
    const uint32_t nchunks = (uint32_t)((shift + L + 15) >> 4);
    const uint4 *gsrc = reinterpret_cast<const uint4 *>(a - shift);
    uint4 *dst = reinterpret_cast<uint4 *>(sm.text);
    for (uint32_t c = lane; c < nchunks; c += 64) dst[c] = gsrc[c];
    sm.rcnt[lane] = 0;
    __syncthreads();
    if (p.debug_stop == 10) continue;                       // profiling only: phase stops 10..13
    const uint8_t *doc = sm.text + shift;
    bool ubad = false, overflow = false, at_end = false, collide = false;
    uint32_t ntok = 0;
    // round insert of each lane's token (have): probe from the key's home slot, linear
    auto insert = [&](uint64_t lo, uint64_t hi, bool have, uint32_t ts32, uint32_t te32) {
      uint32_t slot = dict_hash(lo, hi) >> (32 - kUwSlotBits);
      bool done = !have;
      for (uint32_t r = 0; r < kUwSlots && __any(!done); r++) {
        unsigned long long old = 1;
        if (!done) old = atomicCAS(&sm.klo[slot], 0ull, (unsigned long long)lo);
        const bool won = !done && old == 0;
        if (won) { sm.khi[slot] = hi; sm.kpos[slot] = ts32 | (te32 << 16); }
        asm volatile("" ::: "memory");
        bool match = false;
        if (!done && !won && old == lo) match = sm.khi[slot] == hi;
        if (match && (lo & kLoHashed)) {                    // hashed key: the same term? (kErrCollision if not)
          const uint32_t kp = sm.kpos[slot], ka = kp & 0xFFFFu, kz = kp >> 16;
          collide |= !uc_same_term(doc + ka, kz - ka, doc + ts32, te32 - ts32);
        }
        if (won || match) {
          atomicAdd(&sm.cnt[slot], 1u);
          done = true;
        } else if (!done) {
          slot = (slot + 1) & (kUwSlots - 1);
        }
      }
      overflow |= !done;
    };
    // ---- sparse non-ASCII text (round 5): ASCII words by the wave rules, the
    // islands around non-ASCII bytes by the scanner; tokens inserted 64 a round
    uint32_t nlist = 0;
    const bool sparse = !p.debug_uw_full && shift + (uint32_t)L <= kUwWindow &&
                        uw_sparse_tokens(sm, p, lane, shift, (uint32_t)L, &nlist);
    if (p.debug_stop == 11) continue;
    uint32_t pos = 0, stop = 0;
    if (!sparse) {
      // ---- classes, four consecutive bytes per lane per step
      for (uint32_t i0 = 4 * lane; i0 < L; i0 += 256) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) w |= (i0 + b < L ? (uint32_t)doc[i0 + b] : 0x20u) << (8 * b);
        uint32_t out = 0;
        if ((w & 0x80808080u) == 0) {
#pragma unroll
          for (int b = 0; b < 4; b++) out |= (uint32_t)sm.asc[(w >> (8 * b)) & 0x7Fu] << (8 * b);
        } else {
#pragma unroll
          for (int b = 0; b < 4; b++) {
            const uint32_t x = (w >> (8 * b)) & 0xFFu;
            uint32_t v;
            if (x < 0x80u) v = sm.asc[x];
            else if ((x & 0xC0u) == 0x80u || i0 + b >= L) v = 0xFFu;
            else {
              uint32_t l;
              const uint32_t cp = utf8_decode(doc, L, i0 + b, &l);
              v = cp == kUcBad ? 0xFFu : (uc_class(cp) | ((l - 1) << 5));
            }
            out |= v << (8 * b);
          }
        }
        *reinterpret_cast<uint32_t *>(&sm.cls[i0]) = out;      // bytes past L: never taken
      }
      __syncthreads();
      // ---- slices: lane l scans tokens starting in [cut(l), cut(l + 1))
      const uint64_t seg = (L + 63) >> 6;
      auto cut = [&](uint64_t t) -> uint64_t {
        if (t == 0) return 0;
        uint64_t q = t * seg;
        if (q >= L) return L;
        while (q < L && !uc_split_byte(doc[q - 1])) q++;
        return q;
      };
      pos = (uint32_t)cut(lane);
      stop = (uint32_t)cut(lane + 1);
    }
    // ---- tokens, one per lane per round: the sparse path's list, or the
    // full scan of the lane's slice; each round inserted into the table
    bool active = sparse ? nlist > 0 : pos < stop;
    const uint32_t *tok = reinterpret_cast<const uint32_t *>(sm.cls);
    for (uint32_t t0 = 0; __any(active); t0 += 64) {
      uint64_t lo = 0, hi = 0;
      bool have = false;
      uint32_t ts32 = 0, te32 = 0;
      if (sparse) {
        const uint32_t i = t0 + lane;
        have = i < nlist;
        if (have) {
          const uint32_t e = tok[i];
          ts32 = e & 0xFFFFu;
          te32 = e >> 16;
        }
        active = t0 + 64 < nlist;
      } else if (active) {
        uint32_t p32 = pos;
        have = uc_window_span(sm.cls, sm.tr, (uint32_t)L, &p32, stop, &ts32, &te32, &ubad, &at_end);
        pos = p32;
        active = have;
      }
      if (have) {
        const uint32_t n = te32 - ts32;
        if (n <= 8 && uc_short_ascii_key(sm.text, shift + ts32, n, &lo)) {
          hi = kKeyValid;                                     // most tokens: <= 8 ASCII bytes
          // sparse list: a run of '_' alone is not a token (the scanner never yields one)
          have = lo != (0x5F5F5F5F5F5F5F5Full >> (8 * (8 - n)));
        } else {
          if (sparse && doc[ts32] == '_') {
            bool under = true;
            for (uint32_t j = ts32 + 1; under && j < te32; j++) under = doc[j] == '_';
            have = !under;
          }
          if (have) {
            const uint64_t cutp = uc_token_key(doc, L, ts32, te32, &lo, &hi, p.hash_seed);
            if (cutp < te32) { pos = (uint32_t)cutp; te32 = (uint32_t)cutp; }   // 255-unit cut: rescan from the cut
          }
        }
      }
      ntok += have;
      insert(lo, hi, have, ts32, te32);
    }
    (void)at_end;
    if (collide) set_build_err(p.err, kErrCollision, d);
    // ---- occupied slots, compacted (lane l: slots [16 l, 16 l + 16))
    uint32_t nu;
    {
      uint32_t om = 0;
#pragma unroll
      for (int k = 0; k < (int)(kUwSlots / 64); k++) om |= (uint32_t)(sm.khi[(kUwSlots / 64) * lane + k] != 0) << k;
      const uint32_t c = (uint32_t)__popc(om);
      const uint32_t incl = uw_incl_add(c, lane);
      nu = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      uint32_t at = incl - c;
      while (om) {
        sm.occ[at++] = (uint16_t)((kUwSlots / 64) * lane + (uint32_t)__builtin_ctz(om));
        om &= om - 1;
      }
    }
    __syncthreads();
    if (__any(ubad) || __any(overflow) || nu > kUwMaxTerms || p.debug_stop == 12) {   // wave-uniform: the long path
      if (lane == 0 && p.debug_stop != 12) p.long_list[atomicAdd(p.long_count, 1u)] = d;
      for (uint32_t i = lane; i < nu; i += 64) {
        const uint32_t s = sm.occ[i];
        sm.klo[s] = 0; sm.khi[s] = 0; sm.cnt[s] = 0;
      }
      __syncthreads();
      continue;
    }
    const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)uw_incl_add(ntok, lane), 63);
    // ---- dictionary slots of the occupied entries (4 lookups per lane in flight: two
    // waves per SIMD), range counts
    for (uint32_t h = 0; h * 256 < nu; h++) {
      uint64_t klo[4], khi[4], mine[4];
      bool act[4], cl[4];
      uint32_t g[4], sl[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t i = lane + 64 * (4 * h + k);
        act[k] = i < nu;
        sl[k] = act[k] ? sm.occ[i] : 0u;
        klo[k] = sm.klo[sl[k]];
        khi[k] = sm.khi[sl[k]];
        const uint32_t kp = sm.kpos[sl[k]];
        mine[k] = dict_ref_word(s0 + (kp & 0xFFFFu), (kp >> 16) - (kp & 0xFFFFu));
        if (!act[k]) { klo[k] = 1; khi[k] = kKeyValid; }
      }
      dict_lookup_multi<4>(p.dict, p.cap_mask, klo, khi, act, g, mine, cl);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!act[k]) continue;
        if ((klo[k] & kLoHashed) && !cl[k] && g[k] != kInvalidSlot) dict_verify(p, g[k], mine[k], d);
        uint32_t gs = g[k];
        if (gs == kInvalidSlot) { atomicOr(p.err, kErrCapacity); gs = 0; }
        sm.klo[sl[k]] = gs;
        atomicAdd(&sm.rcnt[gs >> p.range_shift], 1u);
      }
    }
    __syncthreads();
    if (p.debug_stop == 13) {
      for (uint32_t i = lane; i < nu; i += 64) {
        const uint32_t s = sm.occ[i];
        sm.klo[s] = 0; sm.khi[s] = 0; sm.cnt[s] = 0;
      }
      __syncthreads();
      continue;
    }
    // ---- row segments: inclusive ends per range, cursors = exclusive starts
    {
      const uint32_t c = lane < R ? sm.rcnt[lane] : 0u;
      const uint32_t incl = uw_incl_add(c, lane);
      if (lane < R) {
        p.rsplit[(uint64_t)d * R + lane] = incl;
        sm.rcnt[lane] = incl - c;
      }
    }
    __syncthreads();
    const uint64_t base = csr_row_base(p.offsets, src);
    for (uint32_t i = lane; i < nu; i += 64) {
      const uint32_t s = sm.occ[i];
      const uint32_t gs = (uint32_t)sm.klo[s];
      const uint32_t at = atomicAdd(&sm.rcnt[gs >> p.range_shift], 1u);
      csr_put(p, base + at, gs, sm.cnt[s], d);
    }
    __syncthreads();
    for (uint32_t i = lane; i < nu; i += 64) {                // reset the occupied slots for the next document
      const uint32_t s = sm.occ[i];
      sm.klo[s] = 0; sm.khi[s] = 0; sm.cnt[s] = 0;
    }
    if (lane == 0) {
      p.doc_len[d] = len;
      p.doc_nuniq[d] = nu;
      p.doc_norm[d] = (uint8_t)int_to_byte4(len);
      my_dc += len > 0;
      my_ttf += len;
      my_nnz += nu;
    }
    __syncthreads();
    }
  }
  if (lane == 0 && (my_ttf | my_nnz)) {
    atomicAdd(&p.stats[0], my_dc);
    atomicAdd(&p.stats[1], my_ttf);
    atomicAdd(&p.stats[2], my_nnz);
  }
  if (lane == 0 && my_uni) atomicAdd(p.uni_count, my_uni);
}

hipError_t launch_tokenize_uwave(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_uwave, dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Book-sized documents, units with non-ASCII text (round 4).  k_tokenize_chunk
// lists a (document, 2 KB core) unit whose window holds a byte >= 0x80; this
// kernel tokenizes that unit with the Unicode scanner instead of sending the
// whole book to k_tokenize_long.  One wavefront per unit: the window (core +
// context margins) is staged in LDS with per-byte classes; the scan starts at
// a split point (the byte before it is ASCII class OTHER: the scanner's start
// state holds there) at or before the core, lanes take slices between split
// points, and only tokens STARTING in the core are counted (a token crossing
// the core's start belongs to the unit before).  The unit's distinct terms are
// resolved in the dictionary and stored as its bucketed (slot, tf) pair list,
// exactly as k_tokenize_chunk stores an ASCII unit's, for k_long_rows.  A unit
// this cannot take decides its document for the long path (chunk_fail): no
// split point in the leading margin (e.g. unspaced CJK), a token that reaches
// the window's end before the document's, a token over 255 UTF-16 units,
// malformed UTF-8, > kPairWords distinct terms.

// The unit's LDS: a window of at most kPreBytes + kCoreBytes + kPostBytes
// bytes (+ 15 alignment) and a 512-slot term table (a 2 KB core holds at most
// kPairWords distinct terms) — 19 KB, eight workgroups per CU (round 4's first
// form used the 4 KB-window, 1024-slot document layout: 33 KB, four per CU).
constexpr uint32_t kUcWindow = kPreBytes + kCoreBytes + kPostBytes + 16;
constexpr uint32_t kUcSlots = 512;
constexpr uint32_t kUcSlotBits = 9;
struct UcSmem {
  alignas(16) uint8_t text[kUcWindow + 16];
  alignas(16) uint8_t cls[kUcWindow];
  unsigned long long klo[kUcSlots];   // key lo; after the lookup: dictionary slot
  unsigned long long khi[kUcSlots];   // key hi (VALID bit set: occupied)
  uint32_t cnt[kUcSlots];             // tf
  uint32_t kpos[kUcSlots];            // first occurrence: start | end << 16 (window bytes)
  uint16_t occ[kUcSlots];             // occupied slots, compacted
  uint32_t rcnt[64];                  // bucket counts, then cursors
  uint8_t tr[kUwStates * kUwClasses]; // WORD DFA transitions
  uint8_t asc[128];                   // ASCII byte -> scanner class
};

__device__ __forceinline__ void uc_clear_all(UcSmem &sm, uint32_t lane) {
  for (uint32_t s = lane; s < kUcSlots; s += 64) { sm.klo[s] = 0; sm.khi[s] = 0; sm.cnt[s] = 0; }
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) k_tokenize_uchunk(BuildParams p) {
  __shared__ UcSmem sm;
  const uint32_t lane = threadIdx.x;
  // units flagged by k_tokenize_chunk (uchunk_list[u] != 0; *uchunk_count of them)
  if (*p.uchunk_count == 0) return;                         // block-uniform
  for (uint32_t e = lane; e < kUwStates * kUwClasses; e += 64)
    sm.tr[e] = (uint8_t)uc_word_next(e / kUwClasses, e % kUwClasses);
  for (uint32_t e = lane; e < 128; e += 64) sm.asc[e] = (uint8_t)uc_ascii_class(e);
  uc_clear_all(sm, lane);
  __syncthreads();
  for (uint32_t u = blockIdx.x; u < p.n_chunks; u += gridDim.x) {
    if (p.uchunk_list[u] == 0) continue;                    // block-uniform
    const ChunkMeta m = chunk_meta(p, u);
    const uint64_t src = p.live_map ? p.live_map[m.d] : m.d;
    const bool doc_end = m.s0 + m.L == p.offsets[src + 1];  // the window reaches the document's end
    const uint32_t L = (uint32_t)m.L;
    // ---- stage the window (aligned 16 B loads); the table is empty here
    const uint32_t nchunks = (m.shift + L + 15) >> 4;
    const uint4 *gsrc = reinterpret_cast<const uint4 *>(p.text + m.s0 - m.shift);
    uint4 *dst = reinterpret_cast<uint4 *>(sm.text);
    for (uint32_t c = lane; c < nchunks; c += 64) dst[c] = gsrc[c];
    __syncthreads();
    const uint8_t *doc = sm.text + m.shift;
    // ---- classes, four consecutive bytes per lane per step (consecutive lanes
    // on consecutive dwords: no LDS bank conflicts); a char cut by the window's
    // edges is 0xFF: a scan never lands there unless it must fail
    for (uint32_t i0 = 4 * lane; i0 < L; i0 += 256) {
      uint32_t w = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) w |= (i0 + b < L ? (uint32_t)doc[i0 + b] : 0x20u) << (8 * b);
      uint32_t out = 0;
      if ((w & 0x80808080u) == 0) {
#pragma unroll
        for (int b = 0; b < 4; b++) out |= (uint32_t)sm.asc[(w >> (8 * b)) & 0x7Fu] << (8 * b);
      } else {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t x = (w >> (8 * b)) & 0xFFu;
          uint32_t v;
          if (x < 0x80u) v = sm.asc[x];
          else if ((x & 0xC0u) == 0x80u || i0 + b >= L) v = 0xFFu;
          else {
            uint32_t l;
            const uint32_t cp = utf8_decode(doc, L, i0 + b, &l);
            v = cp == kUcBad ? 0xFFu : (uc_class(cp) | ((l - 1) << 5));
          }
          out |= v << (8 * b);
        }
      }
      *reinterpret_cast<uint32_t *>(&sm.cls[i0]) = out;      // bytes past L: never read
    }
    __syncthreads();
    // ---- scan origin: a split point at or before the core (the document's start for its first unit)
    uint32_t start0 = m.core_lo;
    bool fail = false;
    if (m.core_lo > 0) {
      // latest q in [1, core_lo] whose preceding byte is a split byte (lanes test 64 candidates)
      const uint32_t q = m.core_lo - lane;
      const bool ok = lane < m.core_lo && uc_split_byte(doc[q - 1]);
      const uint64_t bm = __ballot(ok);
      if (bm) start0 = m.core_lo - (uint32_t)__builtin_ctzll(bm);
      else fail = true;                                       // no split point in the leading margin
    }
    // ---- slices: lane l scans tokens starting in [cut(l), cut(l + 1)); counted if they start in the core
    const uint32_t hi = m.core_hi;
    const uint32_t seg = (hi - start0 + 63) >> 6;
    auto cut = [&](uint32_t t) -> uint32_t {
      if (t == 0) return start0;
      uint32_t q = start0 + t * seg;
      if (q >= hi) return hi;
      while (q < hi && !uc_split_byte(doc[q - 1])) q++;
      return q;
    };
    uint32_t pos = fail ? hi : cut(lane);
    const uint32_t stop = fail ? hi : cut(lane + 1);
    bool active = pos < stop, ubad = false, overflow = false, at_end = false, collide = false;
    while (__any(active)) {
      uint64_t lo = 0, khv = 0;
      bool have = false;
      uint32_t ts32 = 0, te32 = 0;
      if (active) {
        uint32_t p32 = pos;
        have = uc_window_span(sm.cls, sm.tr, L, &p32, stop, &ts32, &te32, &ubad, &at_end);
        if (have) {
          if (te32 - ts32 <= 8 && uc_short_ascii_key(sm.text, m.shift + ts32, te32 - ts32, &lo)) {
            khv = kKeyValid;                                  // most tokens: <= 8 ASCII bytes
          } else {
            const uint64_t cutp = uc_token_key(doc, L, ts32, te32, &lo, &khv, p.hash_seed);
            if (cutp < te32) overflow = true;                 // > 255 units: the long path cuts it
          }
        }
        pos = p32;
        active = have;
        have = have && ts32 >= m.core_lo;                     // tokens starting in the core only
      }
      uint32_t slot = dict_hash(lo, khv) >> (32 - kUcSlotBits);
      bool done = !have;
      for (uint32_t r = 0; r < kUcSlots && __any(!done); r++) {
        unsigned long long old = 1;
        if (!done) old = atomicCAS(&sm.klo[slot], 0ull, (unsigned long long)lo);
        const bool won = !done && old == 0;
        if (won) { sm.khi[slot] = khv; sm.kpos[slot] = ts32 | (te32 << 16); }
        asm volatile("" ::: "memory");
        bool match = false;
        if (!done && !won && old == lo) match = sm.khi[slot] == khv;
        if (match && (lo & kLoHashed)) {
          const uint32_t kp = sm.kpos[slot], a = kp & 0xFFFFu, z = kp >> 16;
          collide |= !uc_same_term(doc + a, z - a, doc + ts32, te32 - ts32);
        }
        if (won || match) {
          atomicAdd(&sm.cnt[slot], 1u);
          done = true;
        } else if (!done) {
          slot = (slot + 1) & (kUcSlots - 1);
        }
      }
      overflow |= !done;
    }
    if (collide) set_build_err(p.err, kErrCollision, (uint32_t)m.d);
    // ---- occupied slots, compacted (lane l: slots [8 l, 8 l + 8))
    uint32_t nu;
    {
      uint32_t om = 0;
#pragma unroll
      for (int k = 0; k < (int)(kUcSlots / 64); k++) om |= (uint32_t)(sm.khi[(kUcSlots / 64) * lane + k] != 0) << k;
      const uint32_t c = (uint32_t)__popc(om);
      const uint32_t incl = uw_incl_add(c, lane);
      nu = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      uint32_t at = incl - c;
      while (om) {
        sm.occ[at++] = (uint16_t)((kUcSlots / 64) * lane + (uint32_t)__builtin_ctz(om));
        om &= om - 1;
      }
    }
    if (fail || __any(ubad) || __any(overflow) || (__any(at_end) && !doc_end) || nu > kPairWords) {
      if (lane == 0) p.chunk_fail[m.gi] = 1u;                // wave-uniform: the document goes to the long path
      __syncthreads();
      uc_clear_all(sm, lane);
      __syncthreads();
      continue;
    }
    __syncthreads();
    // ---- dictionary slots of the occupied entries (<= 8 per lane, in flight together); bucket counts
    const uint32_t bsh = p.pair_bshift, nb = p.pair_nb, bmask = (1u << bsh) - 1u;
    uint32_t *bcnt = sm.rcnt;                                 // [0, 64) counts, then starts
    bcnt[lane] = 0;
    __syncthreads();
    for (int h = 0; h < 2; h++) {                            // two halves of four (registers: 2 waves / SIMD)
      uint64_t klo[4], khi[4], mine[4];
      bool act[4], cl[4];
      uint32_t g[4], sl[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t i = lane + 64 * (4 * h + k);
        act[k] = i < nu;
        sl[k] = act[k] ? sm.occ[i] : 0u;
        klo[k] = sm.klo[sl[k]];
        khi[k] = sm.khi[sl[k]];
        const uint32_t kp = sm.kpos[sl[k]];
        mine[k] = dict_ref_word(m.s0 + (kp & 0xFFFFu), (kp >> 16) - (kp & 0xFFFFu));
        if (!act[k]) { klo[k] = 1; khi[k] = kKeyValid; }
      }
      if (!__any(act[0])) break;                              // wave-uniform: no terms left
      dict_lookup_multi<4>(p.dict, p.cap_mask, klo, khi, act, g, mine, cl);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (!act[k]) continue;
        if ((klo[k] & kLoHashed) && !cl[k] && g[k] != kInvalidSlot) dict_verify(p, g[k], mine[k], (uint32_t)m.d);
        uint32_t gs = g[k];
        if (gs == kInvalidSlot) { atomicOr(p.err, kErrCapacity); gs = 0; }
        sm.klo[sl[k]] = gs;
        atomicAdd(&bcnt[gs >> bsh], 1u);
      }
    }
    __syncthreads();
    // ---- the unit's pair list, counting-sorted by bucket (k_tokenize_chunk's format)
    {
      const uint32_t c = lane < nb ? bcnt[lane] : 0u;
      const uint32_t incl = uw_incl_add(c, lane);
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      uint32_t *ub = p.pair_ub + (uint64_t)u * (nb + 1);
      if (lane < nb) ub[lane] = incl - c;
      if (lane == 0) ub[nb] = total;
      __syncthreads();
      if (lane < nb) bcnt[lane] = incl - c;                   // cursors
      __syncthreads();
      uint32_t *stage = reinterpret_cast<uint32_t *>(sm.cls);  // classes are dead here (kPairWords words fit)
      for (uint32_t i = lane; i < nu; i += 64) {
        const uint32_t s = sm.occ[i];
        const uint32_t gs = (uint32_t)sm.klo[s];
        const uint32_t at = atomicAdd(&bcnt[gs >> bsh], 1u);
        stage[at] = ((gs & bmask) << kPairTfBits) | sm.cnt[s];
      }
      __syncthreads();
      uint32_t *pr = p.pairs + (uint64_t)u * kPairWords;
      for (uint32_t i = lane; i < total; i += 64) pr[i] = stage[i];
      // reset the occupied slots for the next unit
      for (uint32_t i = lane; i < nu; i += 64) {
        const uint32_t s = sm.occ[i];
        sm.klo[s] = 0; sm.khi[s] = 0; sm.cnt[s] = 0;
      }
    }
    __syncthreads();
  }
}

hipError_t launch_tokenize_uchunk(const BuildParams &p, int grid, hipStream_t s) {
  hipLaunchKernelGGL(k_tokenize_uchunk, dim3(grid), dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace tfidf
