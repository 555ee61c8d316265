/*
 * tfidf_oracle.c — CPU ORACLE (test infrastructure; see tfidf_oracle.h).
 *
 * Restates, single-threaded and in Java's float/double operation order:
 *  - Lucene 9.8.0 StandardTokenizer (JFlex UAX#29 word-break grammar, full
 *    Unicode: letters, digits, Katakana, Hebrew quotes, Complex_Context runs,
 *    Han / Hiragana single chars, emoji; ASCII text takes a byte-rule fast
 *    path that tests check against the Unicode rules), maxTokenLength 255
 *    (UTF-16 units; longer tokens are chopped and scanning restarts at the
 *    chop point), LowerCaseFilter (JDK 17 Character.toLowerCase), empty StopFilter
 *    (StandardAnalyzer, constructed at Worker.java:71 and :225).
 *  - IndexingChain inversion per doc (Worker.java:218): TF per term, field
 *    length = #tokens, norm = SmallFloat.intToByte4(length) (0 when empty).
 *  - Collection stats: docFreq per term, docCount = #docs with >= 1 token,
 *    sumTotalTermFreq.
 *  - QueryParser.escape + parse with default OR (Worker.java:226-227),
 *    BooleanQuery SHOULD de-duplication (boost = occurrence count).
 *  - BM25Similarity(k1 = 1.2f, b = 0.75f) weight/scorer; disjunction sums
 *    per-term float scores in double and rounds once (WANDScorer/
 *    BooleanScorer); TopScoreDocCollector order (score desc, doc asc);
 *    searcher.search(q, Integer.MAX_VALUE) -> all hits (Worker.java:230).
 *  - Leader.start merge (Leader.java:73-88): Double::sum per name, TreeMap
 *    order.
 * Compile with -ffp-contract=off and no fast-math (SSE float = Java float).
 */
#define _POSIX_C_SOURCE 200809L
#include "tfidf_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* Character classes: Unicode Word_Break property restricted to ASCII. */
enum { C_O = 0, C_L, C_D, C_U, C_ML, C_MNL, C_MN };

static int wb_class(uint8_t c) {
  if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) return C_L;  /* ALetter */
  if (c >= '0' && c <= '9') return C_D;                              /* Numeric */
  switch (c) {
    case '_': return C_U;              /* ExtendNumLet */
    case ':': return C_ML;             /* MidLetter */
    case '.': case '\'': return C_MNL; /* MidNumLet, Single_Quote (MidNumLetQ) */
    case ',': case ';': return C_MN;   /* MidNum */
    default: return C_O;
  }
}

/* Is byte i part of a word segment, given scanning restarted at lo?
 * WB5/8/9/10/13a/13b join letters, digits and '_' pairwise; WB6/WB7 join
 * L (MidLetter|MidNumLetQ) L; WB11/WB12 join D (MidNum|MidNumLetQ) D. */
static int is_word(const uint8_t *s, uint64_t lo, uint64_t n, uint64_t i) {
  int c = wb_class(s[i]);
  if (c == C_L || c == C_D || c == C_U) return 1;
  if (c == C_O || i == lo || i + 1 >= n) return 0;
  int a = wb_class(s[i - 1]), z = wb_class(s[i + 1]);
  if ((c == C_ML || c == C_MNL) && a == C_L && z == C_L) return 1;
  if ((c == C_MN || c == C_MNL) && a == C_D && z == C_D) return 1;
  return 0;
}

int64_t orc_tokenize_unicode(const uint8_t *s, uint64_t n, uint32_t max_len, uint32_t *starts, uint32_t *lens,
                             uint64_t cap);

int64_t orc_tokenize(const uint8_t *s, uint64_t n, uint32_t max_len,
                     uint32_t *starts, uint32_t *lens, uint64_t cap) {
  for (uint64_t i = 0; i < n; i++)
    if (s[i] >= 0x80) return orc_tokenize_unicode(s, n, max_len, starts, lens, cap);
  if (max_len == 0) max_len = 255;
  uint64_t lo = 0, i = 0;
  int64_t cnt = 0;
  while (i < n) {
    if (!is_word(s, lo, n, i)) { i++; continue; }
    uint64_t j = i;
    int has_ld = 0;
    while (j < n && is_word(s, lo, n, j)) {
      int c = wb_class(s[j]);
      has_ld |= (c == C_L || c == C_D);
      j++;
    }
    if (!has_ld) { i = j; continue; }          /* "___" alone is not a token */
    if (j - i > max_len) {                      /* chop + rescan from the cut */
      if ((uint64_t)cnt < cap) { starts[cnt] = (uint32_t)i; lens[cnt] = max_len; }
      cnt++;
      lo = i + max_len;
      i = lo;
      continue;
    }
    if ((uint64_t)cnt < cap) { starts[cnt] = (uint32_t)i; lens[cnt] = (uint32_t)(j - i); }
    cnt++;
    i = j;
  }
  return cnt;
}

/* ------------------------------------------------------------------ */
/* Full-Unicode StandardTokenizer (Lucene 9.8.0 StandardTokenizerImpl, JFlex
 * `%unicode 9.0`), restated by LOCAL JOIN RULES between adjacent units (the
 * product scans with a longest-match DFA instead, unicode_scan.h; the Python
 * transcription of the JFlex grammar in tests/ pins both).  A unit is a head
 * char plus its trailing Extend/Format/ZWJ chars (WB4); a head of class OTHER
 * does not take extenders (JFlex's [^] rule consumes one char), so an
 * extender after it is its own unit, skipped — or, if it is a Complex_Context
 * (Line_Break SA) mark, the start of an SA run. */
#include "unicode_props.h"

enum { UC_OTHER = 0, UC_AL, UC_HL, UC_NU, UC_KA, UC_EX, UC_ML, UC_MNL, UC_MN, UC_SQ, UC_DQ, UC_EXT, UC_EXT_SA,
       UC_ZWJ, UC_SA, UC_HAN, UC_HIRA, UC_RI, UC_EMO };

static int uc_cls(uint32_t cp) {
  int lo = 0, hi = UC_NRANGES - 1;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    if (cp < uc_ranges[mid][0]) hi = mid - 1;
    else if (cp > uc_ranges[mid][1]) lo = mid + 1;
    else return (int)uc_ranges[mid][2];
  }
  return UC_OTHER;
}
static uint32_t uc_tolower(uint32_t cp) {   /* JDK 17 Character.toLowerCase(int) */
  int lo = 0, hi = UC_NLOWER - 1;
  while (lo <= hi) {
    int mid = (lo + hi) / 2;
    if (cp < uc_lower[mid][0]) hi = mid - 1;
    else if (cp > uc_lower[mid][0]) lo = mid + 1;
    else return uc_lower[mid][1];
  }
  return cp;
}
static int is_ext(int c) { return c == UC_EXT || c == UC_EXT_SA || c == UC_ZWJ; }
static int is_ahl(int c) { return c == UC_AL || c == UC_HL; }
static int is_midlet(int c) { return c == UC_ML || c == UC_MNL || c == UC_SQ; }
static int is_midnum(int c) { return c == UC_MN || c == UC_MNL || c == UC_SQ; }
static int is_wordish(int c) { return c == UC_AL || c == UC_HL || c == UC_NU || c == UC_KA || c == UC_EX; }

/* RFC 3629 strict decode of the whole text; -1 on malformed input. */
static int64_t utf8_all(const uint8_t *s, uint64_t n, uint32_t *cps, uint32_t *offs) {
  uint64_t i = 0, k = 0;
  while (i < n) {
    uint32_t b = s[i], cp, need, min;
    if (b < 0x80) { cp = b; need = 0; min = 0; }
    else if ((b & 0xE0) == 0xC0) { cp = b & 0x1F; need = 1; min = 0x80; }
    else if ((b & 0xF0) == 0xE0) { cp = b & 0x0F; need = 2; min = 0x800; }
    else if ((b & 0xF8) == 0xF0) { cp = b & 0x07; need = 3; min = 0x10000; }
    else return -1;
    if (i + need >= n && need) return -1;
    for (uint32_t t = 1; t <= need; t++) {
      uint32_t c = s[i + t];
      if ((c & 0xC0) != 0x80) return -1;
      cp = (cp << 6) | (c & 0x3F);
    }
    if (cp < min || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return -1;
    cps[k] = cp;
    offs[k] = (uint32_t)i;
    k++;
    i += need + 1;
  }
  offs[k] = (uint32_t)n;
  return (int64_t)k;
}

typedef struct { uint64_t a, b; int c; int zwj; } uc_unit_t;   /* cp range [a, b), head class */

/* unit at code point index i (head never an absorbed extender) */
static uc_unit_t unit_at(const int *cls, uint64_t m, uint64_t i) {
  uc_unit_t u;
  u.a = i; u.c = cls[i]; u.zwj = 0;
  uint64_t j = i + 1;
  if (u.c == UC_EXT_SA) u.c = UC_SA;                 /* orphan SA mark: an SA head */
  if (u.c != UC_OTHER && u.c != UC_EXT && u.c != UC_ZWJ)
    while (j < m && is_ext(cls[j])) { u.zwj = cls[j] == UC_ZWJ; j++; }
  u.b = j;
  return u;
}

/* do units x (with predecessor w, or w.c = -1) and y (successor z, or -1) join in one WORD token? */
static int word_join(int w, int x, int y, int z) {
  if (x == UC_EX && is_wordish(y)) return 1;                         /* WB13b + ENL runs */
  if (is_wordish(x) && y == UC_EX) return 1;                         /* WB13a */
  if ((is_ahl(x) || x == UC_NU) && (is_ahl(y) || y == UC_NU)) return 1;  /* WB5, WB8, WB9, WB10 */
  if (x == UC_KA && y == UC_KA) return 1;                            /* WB13 */
  if (x == UC_HL && y == UC_SQ) return 1;                            /* WB7a */
  if (x == UC_SQ && w == UC_HL && (is_ahl(y) || y == UC_NU || y == UC_EX)) return 1;  /* Hgrp then a group */
  if (is_ahl(x) && is_midlet(y) && is_ahl(z)) return 1;              /* WB6 */
  if (is_midlet(x) && is_ahl(w) && is_ahl(y)) return 1;              /* WB7 */
  if (x == UC_NU && is_midnum(y) && z == UC_NU) return 1;            /* WB12 */
  if (is_midnum(x) && w == UC_NU && y == UC_NU) return 1;            /* WB11 */
  if (x == UC_HL && y == UC_DQ && z == UC_HL) return 1;              /* WB7b */
  if (x == UC_DQ && w == UC_HL && y == UC_HL) return 1;              /* WB7c */
  return 0;
}

int64_t orc_tokenize_unicode(const uint8_t *s, uint64_t n, uint32_t max_len, uint32_t *starts, uint32_t *lens,
                             uint64_t cap) {
  if (max_len == 0) max_len = 255;
  uint32_t *cps = (uint32_t *)malloc((n + 1) * 4), *offs = (uint32_t *)malloc((n + 1) * 4);
  int *cls = (int *)malloc((n + 1) * sizeof(int));
  if (!cps || !offs || !cls) { free(cps); free(offs); free(cls); return ORC_E_NOMEM; }
  int64_t m = utf8_all(s, n, cps, offs);
  if (m < 0) { free(cps); free(offs); free(cls); return ORC_E_UNSUPPORTED; }
  for (int64_t i = 0; i < m; i++) cls[i] = uc_cls(cps[i]);
  int64_t cnt = 0;
  uint64_t i = 0;
#define EMIT(A, B)                                                                    \
  do {                                                                                \
    uint64_t a_ = (A), b_ = (B), u16_ = 0, e_ = a_;                                   \
    while (e_ < b_ && u16_ + (cps[e_] >= 0x10000 ? 2 : 1) <= max_len) u16_ += (cps[e_++] >= 0x10000 ? 2 : 1); \
    if ((uint64_t)cnt < cap) { starts[cnt] = offs[a_]; lens[cnt] = offs[e_] - offs[a_]; } \
    cnt++;                                                                            \
    i = e_;                                                                           \
  } while (0)
  while (i < (uint64_t)m) {
    uc_unit_t u = unit_at(cls, (uint64_t)m, i);
    if (is_wordish(u.c)) {
      /* maximal run of joined units */
      uc_unit_t w = {0, 0, -1, 0}, x = u;
      int core = x.c != UC_EX;
      uint64_t end = x.b;
      while (x.b < (uint64_t)m) {
        uc_unit_t y = unit_at(cls, (uint64_t)m, x.b);
        int z = -1;
        if (y.b < (uint64_t)m) z = unit_at(cls, (uint64_t)m, y.b).c;
        if (!word_join(w.c, x.c, y.c, z)) break;
        w = x; x = y;
        core |= x.c != UC_EX;
        end = x.b;
      }
      if (core) { EMIT(u.a, end); continue; }
      /* ENL-only run: JFlex skips char by char; an absorbed SA mark starts an SA run */
      uint64_t k = u.a + 1;
      while (k < end && cls[k] != UC_EXT_SA) k++;
      i = k;
      continue;
    }
    if (u.c == UC_SA) {
      uint64_t e = u.b;
      while (e < (uint64_t)m && (cls[e] == UC_SA || is_ext(cls[e]))) e++;
      EMIT(u.a, e);
      continue;
    }
    if (u.c == UC_HAN || u.c == UC_HIRA) { EMIT(u.a, u.b); continue; }
    if (u.c == UC_EMO) {
      uc_unit_t x = u;
      while (x.zwj && x.b < (uint64_t)m) {
        uc_unit_t y = unit_at(cls, (uint64_t)m, x.b);
        if (y.c != UC_EMO) break;
        x = y;
      }
      EMIT(u.a, x.b);
      continue;
    }
    if (u.c == UC_RI && u.b < (uint64_t)m) {
      uc_unit_t y = unit_at(cls, (uint64_t)m, u.b);
      if (y.c == UC_RI) { EMIT(u.a, y.b); continue; }
    }
    i = i + 1;                                        /* [^] */
  }
#undef EMIT
  free(cps); free(offs); free(cls);
  return cnt;
}

/* LowerCaseFilter on one token: UTF-8 -> UTF-8 of Character.toLowerCase per
 * code point.  dst needs 2 * len bytes.  Returns the output length. */
uint64_t orc_lower_utf8(const uint8_t *src, uint64_t len, uint8_t *dst) {
  uint64_t i = 0, o = 0;
  while (i < len) {
    uint32_t b = src[i], cp, need;
    if (b < 0x80) { cp = b; need = 0; }
    else if ((b & 0xE0) == 0xC0) { cp = b & 0x1F; need = 1; }
    else if ((b & 0xF0) == 0xE0) { cp = b & 0x0F; need = 2; }
    else { cp = b & 0x07; need = 3; }
    for (uint32_t t = 1; t <= need; t++) cp = (cp << 6) | (src[i + t] & 0x3F);
    i += need + 1;
    uint32_t lc = cp < 0x80 ? ((cp >= 'A' && cp <= 'Z') ? cp + 32 : cp) : uc_tolower(cp);
    if (lc < 0x80) dst[o++] = (uint8_t)lc;
    else if (lc < 0x800) { dst[o++] = (uint8_t)(0xC0 | (lc >> 6)); dst[o++] = (uint8_t)(0x80 | (lc & 0x3F)); }
    else if (lc < 0x10000) {
      dst[o++] = (uint8_t)(0xE0 | (lc >> 12)); dst[o++] = (uint8_t)(0x80 | ((lc >> 6) & 0x3F));
      dst[o++] = (uint8_t)(0x80 | (lc & 0x3F));
    } else {
      dst[o++] = (uint8_t)(0xF0 | (lc >> 18)); dst[o++] = (uint8_t)(0x80 | ((lc >> 12) & 0x3F));
      dst[o++] = (uint8_t)(0x80 | ((lc >> 6) & 0x3F)); dst[o++] = (uint8_t)(0x80 | (lc & 0x3F));
    }
  }
  return o;
}

/* ------------------------------------------------------------------ */
/* SmallFloat (org.apache.lucene.util.SmallFloat) */
static int bitlen64(uint64_t v) { int n = 0; while (v) { n++; v >>= 1; } return n; }

static int32_t long_to_int4(int64_t i) {
  int nb = bitlen64((uint64_t)i);
  if (nb < 4) return (int32_t)i;
  int sh = nb - 4;
  return (int32_t)(((i >> sh) & 7) | ((int64_t)(sh + 1) << 3));
}
static int64_t int4_to_long(int32_t e) {
  int64_t bits = e & 7;
  int sh = (e >> 3) - 1;
  if (sh == -1) return bits;
  return (bits | 8) << sh;
}
#define NUM_FREE_VALUES 24 /* 255 - longToInt4(Integer.MAX_VALUE) */

uint8_t orc_int_to_byte4(int32_t i) {
  if (i < NUM_FREE_VALUES) return (uint8_t)i;
  return (uint8_t)(NUM_FREE_VALUES + long_to_int4((int64_t)i - NUM_FREE_VALUES));
}
int32_t orc_byte4_to_int(uint8_t b) {
  int32_t i = b;
  if (i < NUM_FREE_VALUES) return i;
  return (int32_t)(NUM_FREE_VALUES + int4_to_long(i - NUM_FREE_VALUES));
}

/* ------------------------------------------------------------------ */
/* BM25Similarity (9.8.0) in Java operation order. */
float orc_idf(uint64_t doc_freq, uint64_t doc_count) {
  double x = ((double)((int64_t)doc_count - (int64_t)doc_freq) + 0.5) / ((double)doc_freq + 0.5);
  return (float)log(1.0 + x);
}
float orc_avgdl(uint64_t sum_ttf, uint64_t doc_count) {
  return (float)((double)sum_ttf / (double)doc_count);
}
void orc_norm_cache(float k1, float b, float avgdl, float cache[256]) {
  for (int i = 0; i < 256; i++) {
    float len = (float)orc_byte4_to_int((uint8_t)i);
    volatile float t1 = 1.0f - b;
    volatile float t2 = b * len;
    volatile float t3 = t2 / avgdl;
    volatile float t4 = t1 + t3;
    volatile float t5 = k1 * t4;
    cache[i] = 1.0f / t5;
  }
}
float orc_bm25(float weight, uint32_t tf, float norm_inverse) {
  volatile float f = (float)tf;
  volatile float t = f * norm_inverse;
  volatile float u = 1.0f + t;
  volatile float v = weight / u;
  return weight - v;
}

/* ------------------------------------------------------------------ */
/* Small string-keyed open-addressing table. */
typedef struct {
  char *arena;
  uint64_t arena_len, arena_cap;
  uint64_t *off;    /* per term: arena offset */
  uint32_t *len;    /* per term: length */
  uint64_t n, cap_terms;
  int64_t *slots;   /* -1 = empty, else term id */
  uint64_t nslots;
} strtab;

static uint64_t fnv1a(const uint8_t *p, uint64_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint64_t i = 0; i < n; i++) { h ^= p[i]; h *= 1099511628211ull; }
  return h;
}

static int st_init(strtab *t) {
  memset(t, 0, sizeof(*t));
  t->nslots = 1024;
  t->slots = (int64_t *)malloc(t->nslots * sizeof(int64_t));
  if (!t->slots) return ORC_E_NOMEM;
  for (uint64_t i = 0; i < t->nslots; i++) t->slots[i] = -1;
  return ORC_OK;
}
static void st_free(strtab *t) {
  free(t->arena); free(t->off); free(t->len); free(t->slots);
  memset(t, 0, sizeof(*t));
}
static const char *st_str(const strtab *t, uint64_t id) { return t->arena + t->off[id]; }

static int64_t st_find(const strtab *t, const uint8_t *p, uint64_t n) {
  uint64_t m = t->nslots - 1, h = fnv1a(p, n) & m;
  for (;;) {
    int64_t id = t->slots[h];
    if (id < 0) return -1;
    if (t->len[id] == n && memcmp(st_str(t, (uint64_t)id), p, n) == 0) return id;
    h = (h + 1) & m;
  }
}

static int st_grow(strtab *t) {
  uint64_t ns = t->nslots * 2;
  int64_t *s = (int64_t *)malloc(ns * sizeof(int64_t));
  if (!s) return ORC_E_NOMEM;
  for (uint64_t i = 0; i < ns; i++) s[i] = -1;
  for (uint64_t id = 0; id < t->n; id++) {
    uint64_t h = fnv1a((const uint8_t *)st_str(t, id), t->len[id]) & (ns - 1);
    while (s[h] >= 0) h = (h + 1) & (ns - 1);
    s[h] = (int64_t)id;
  }
  free(t->slots);
  t->slots = s;
  t->nslots = ns;
  return ORC_OK;
}

static int64_t st_insert(strtab *t, const uint8_t *p, uint64_t n) {
  int64_t id = st_find(t, p, n);
  if (id >= 0) return id;
  if ((t->n + 1) * 2 > t->nslots && st_grow(t) != ORC_OK) return ORC_E_NOMEM;
  if (t->n == t->cap_terms) {
    uint64_t nc = t->cap_terms ? t->cap_terms * 2 : 256;
    uint64_t *o = (uint64_t *)realloc(t->off, nc * sizeof(uint64_t));
    if (!o) return ORC_E_NOMEM;
    t->off = o;
    uint32_t *l = (uint32_t *)realloc(t->len, nc * sizeof(uint32_t));
    if (!l) return ORC_E_NOMEM;
    t->len = l;
    t->cap_terms = nc;
  }
  if (t->arena_len + n + 1 > t->arena_cap) {
    uint64_t nc = t->arena_cap ? t->arena_cap * 2 : 4096;
    while (nc < t->arena_len + n + 1) nc *= 2;
    char *a = (char *)realloc(t->arena, nc);
    if (!a) return ORC_E_NOMEM;
    t->arena = a;
    t->arena_cap = nc;
  }
  memcpy(t->arena + t->arena_len, p, n);
  t->arena[t->arena_len + n] = 0;
  id = (int64_t)t->n++;
  t->off[id] = t->arena_len;
  t->len[id] = (uint32_t)n;
  t->arena_len += n + 1;
  uint64_t m = t->nslots - 1, h = fnv1a(p, n) & m;
  while (t->slots[h] >= 0) h = (h + 1) & m;
  t->slots[h] = id;
  return id;
}

/* ------------------------------------------------------------------ */
typedef struct { uint32_t doc, tf; } posting;

typedef struct {
  uint8_t *key; uint64_t key_len;
  uint8_t *text; uint64_t text_len;
  int live;
} stored_doc;

struct orc_index {
  float k1, b;
  stored_doc *docs; uint64_t ndocs, docs_cap;     /* staged (incl. replaced) */
  /* committed state */
  uint64_t *live;  uint64_t nlive;                /* committed doc -> staged idx */
  uint32_t *doc_len; uint8_t *doc_norm;
  uint64_t *dt_off; uint32_t *dt_term; uint32_t *dt_tf; /* per-doc terms, sorted */
  strtab terms;
  uint64_t *df;                                   /* per term */
  posting **plist; uint64_t *plen;                /* postings in doc order */
  uint64_t doc_count, sum_ttf;
  uint64_t *malformed; uint64_t n_malformed;      /* committed docs not valid UTF-8 */
  /* global override */
  uint64_t g_doc_count, g_sum_ttf;
  strtab g_terms; uint64_t *g_df; uint64_t g_df_cap;
  int committed;
};

orc_index *orc_create(float k1, float b) {
  orc_index *ix = (orc_index *)calloc(1, sizeof(orc_index));
  if (!ix) return NULL;
  ix->k1 = k1; ix->b = b;
  st_init(&ix->terms);
  st_init(&ix->g_terms);
  return ix;
}

static void free_committed(orc_index *ix) {
  free(ix->live); free(ix->doc_len); free(ix->doc_norm); free(ix->malformed);
  ix->malformed = NULL; ix->n_malformed = 0;
  free(ix->dt_off); free(ix->dt_term); free(ix->dt_tf);
  if (ix->plist) for (uint64_t t = 0; t < ix->terms.n; t++) free(ix->plist[t]);
  free(ix->plist); free(ix->plen); free(ix->df);
  st_free(&ix->terms);
  st_init(&ix->terms);
  ix->live = NULL; ix->doc_len = NULL; ix->doc_norm = NULL;
  ix->dt_off = NULL; ix->dt_term = NULL; ix->dt_tf = NULL;
  ix->plist = NULL; ix->plen = NULL; ix->df = NULL;
  ix->committed = 0;
}

void orc_destroy(orc_index *ix) {
  if (!ix) return;
  free_committed(ix);
  st_free(&ix->terms);
  st_free(&ix->g_terms);
  free(ix->g_df);
  for (uint64_t i = 0; i < ix->ndocs; i++) { free(ix->docs[i].key); free(ix->docs[i].text); }
  free(ix->docs);
  free(ix);
}

int orc_add_doc(orc_index *ix, const uint8_t *key, uint64_t key_len,
                const uint8_t *text, uint64_t n) {
  if (!ix) return ORC_E_ARG;
  for (uint64_t i = 0; i < ix->ndocs; i++)
    if (ix->docs[i].live && ix->docs[i].key_len == key_len &&
        memcmp(ix->docs[i].key, key, key_len) == 0)
      ix->docs[i].live = 0;                     /* delete-by-term */
  if (ix->ndocs == ix->docs_cap) {
    uint64_t nc = ix->docs_cap ? ix->docs_cap * 2 : 64;
    stored_doc *d = (stored_doc *)realloc(ix->docs, nc * sizeof(stored_doc));
    if (!d) return ORC_E_NOMEM;
    ix->docs = d; ix->docs_cap = nc;
  }
  stored_doc *d = &ix->docs[ix->ndocs++];
  d->key = (uint8_t *)malloc(key_len + 1);
  d->text = (uint8_t *)malloc(n + 1);
  if (!d->key || !d->text) return ORC_E_NOMEM;
  memcpy(d->key, key, key_len); d->key_len = key_len;
  memcpy(d->text, text, n); d->text_len = n;
  d->live = 1;
  return ORC_OK;
}


static int cmp_term_ids(const void *a, const void *b, void *ctx) {
  const strtab *t = (const strtab *)ctx;
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return strcmp(st_str(t, x), st_str(t, y));
}

/* Per-document term order (bytes): bottom-up merge sort of (term id, tf)
 * pairs keyed by the term strings (qsort_r is a GNU extension; the context
 * is passed explicitly so concurrent indexes on several threads are safe). */
static void sort_terms(uint32_t *ids, uint32_t *tfs, uint64_t n, const strtab *t) {
  if (n < 2) return;
  uint32_t *bi = (uint32_t *)malloc(n * 4), *bt = (uint32_t *)malloc(n * 4);
  if (!bi || !bt) {                                  /* out of memory: insertion sort in place */
    free(bi); free(bt);
    for (uint64_t i = 1; i < n; i++) {
      uint32_t a = ids[i], f = tfs[i];
      uint64_t j = i;
      while (j > 0 && cmp_term_ids(&ids[j - 1], &a, (void *)t) > 0) { ids[j] = ids[j - 1]; tfs[j] = tfs[j - 1]; j--; }
      ids[j] = a; tfs[j] = f;
    }
    return;
  }
  uint32_t *si = ids, *st = tfs, *di = bi, *dt = bt;
  for (uint64_t w = 1; w < n; w *= 2) {
    for (uint64_t lo = 0; lo < n; lo += 2 * w) {
      uint64_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
      uint64_t a = lo, b = mid, o = lo;
      while (a < mid && b < hi) {
        if (cmp_term_ids(&si[b], &si[a], (void *)t) < 0) { di[o] = si[b]; dt[o] = st[b]; b++; }
        else { di[o] = si[a]; dt[o] = st[a]; a++; }
        o++;
      }
      while (a < mid) { di[o] = si[a]; dt[o] = st[a]; a++; o++; }
      while (b < hi) { di[o] = si[b]; dt[o] = st[b]; b++; o++; }
    }
    uint32_t *x = si; si = di; di = x;
    x = st; st = dt; dt = x;
  }
  if (si != ids) { memcpy(ids, si, n * 4); memcpy(tfs, st, n * 4); }
  free(bi); free(bt);
}

int orc_commit(orc_index *ix) {
  if (!ix) return ORC_E_ARG;
  free_committed(ix);
  uint64_t nlive = 0;
  for (uint64_t i = 0; i < ix->ndocs; i++) nlive += ix->docs[i].live;
  ix->live = (uint64_t *)malloc((nlive + 1) * sizeof(uint64_t));
  ix->doc_len = (uint32_t *)calloc(nlive + 1, sizeof(uint32_t));
  ix->doc_norm = (uint8_t *)calloc(nlive + 1, 1);
  ix->dt_off = (uint64_t *)calloc(nlive + 1, sizeof(uint64_t));
  if (!ix->live || !ix->doc_len || !ix->doc_norm || !ix->dt_off) return ORC_E_NOMEM;
  uint64_t k = 0;
  for (uint64_t i = 0; i < ix->ndocs; i++) if (ix->docs[i].live) ix->live[k++] = i;
  ix->nlive = nlive;

  uint64_t dt_cap = 1024, dt_n = 0;
  ix->dt_term = (uint32_t *)malloc(dt_cap * sizeof(uint32_t));
  ix->dt_tf = (uint32_t *)malloc(dt_cap * sizeof(uint32_t));
  uint64_t tok_cap = 1024;
  uint32_t *st = (uint32_t *)malloc(tok_cap * 4), *ln = (uint32_t *)malloc(tok_cap * 4);
  uint64_t last_cap = 0;
  int64_t *last_doc = NULL; uint64_t *slot_of = NULL;
  uint8_t *lbuf = (uint8_t *)malloc(2048);
  if (!ix->dt_term || !ix->dt_tf || !st || !ln || !lbuf) return ORC_E_NOMEM;
  ix->doc_count = 0; ix->sum_ttf = 0;

  for (uint64_t d = 0; d < nlive; d++) {
    const stored_doc *sd = &ix->docs[ix->live[d]];
    int64_t nt = orc_tokenize(sd->text, sd->text_len, 255, st, ln, tok_cap);
    if (nt == ORC_E_UNSUPPORTED) {
      /* Files.readString throws MalformedInputException (Worker.java:199-201);
       * the text then comes from Tika (text = "" when Tika fails), which is not rebuilt: the
       * document is indexed with an empty field and listed. */
      if (!ix->malformed) ix->malformed = (uint64_t *)malloc(nlive * sizeof(uint64_t));
      if (!ix->malformed) return ORC_E_NOMEM;
      ix->malformed[ix->n_malformed++] = d;
      nt = 0;
    }
    if (nt < 0) return (int)nt;
    if ((uint64_t)nt > tok_cap) {
      tok_cap = (uint64_t)nt;
      st = (uint32_t *)realloc(st, tok_cap * 4); ln = (uint32_t *)realloc(ln, tok_cap * 4);
      if (!st || !ln) return ORC_E_NOMEM;
      orc_tokenize(sd->text, sd->text_len, 255, st, ln, tok_cap);
    }
    uint64_t row0 = dt_n;
    ix->dt_off[d] = row0;
    for (int64_t t = 0; t < nt; t++) {
      const uint64_t ll = orc_lower_utf8(sd->text + st[t], ln[t], lbuf);
      int64_t id = st_insert(&ix->terms, lbuf, ll);
      if (id < 0) return ORC_E_NOMEM;
      if ((uint64_t)id >= last_cap) {
        uint64_t nc = last_cap ? last_cap * 2 : 1024;
        while (nc <= (uint64_t)id) nc *= 2;
        last_doc = (int64_t *)realloc(last_doc, nc * sizeof(int64_t));
        slot_of = (uint64_t *)realloc(slot_of, nc * sizeof(uint64_t));
        if (!last_doc || !slot_of) return ORC_E_NOMEM;
        for (uint64_t z = last_cap; z < nc; z++) last_doc[z] = -1;
        last_cap = nc;
      }
      if (last_doc[id] != (int64_t)d) {
        last_doc[id] = (int64_t)d;
        if (dt_n == dt_cap) {
          dt_cap *= 2;
          ix->dt_term = (uint32_t *)realloc(ix->dt_term, dt_cap * 4);
          ix->dt_tf = (uint32_t *)realloc(ix->dt_tf, dt_cap * 4);
          if (!ix->dt_term || !ix->dt_tf) return ORC_E_NOMEM;
        }
        slot_of[id] = dt_n;
        ix->dt_term[dt_n] = (uint32_t)id;
        ix->dt_tf[dt_n] = 0;
        dt_n++;
      }
      ix->dt_tf[slot_of[id]]++;
    }
    sort_terms(ix->dt_term + row0, ix->dt_tf + row0, dt_n - row0, &ix->terms);
    ix->doc_len[d] = (uint32_t)nt;
    ix->doc_norm[d] = orc_int_to_byte4((int32_t)nt);  /* 0 for an empty field */
    if (nt > 0) ix->doc_count++;
    ix->sum_ttf += (uint64_t)nt;
  }
  ix->dt_off[nlive] = dt_n;
  free(st); free(ln); free(last_doc); free(slot_of); free(lbuf);

  uint64_t V = ix->terms.n;
  ix->df = (uint64_t *)calloc(V + 1, sizeof(uint64_t));
  ix->plen = (uint64_t *)calloc(V + 1, sizeof(uint64_t));
  ix->plist = (posting **)calloc(V + 1, sizeof(posting *));
  if (!ix->df || !ix->plen || !ix->plist) return ORC_E_NOMEM;
  for (uint64_t e = 0; e < dt_n; e++) ix->df[ix->dt_term[e]]++;
  for (uint64_t t = 0; t < V; t++) {
    ix->plist[t] = (posting *)malloc((ix->df[t] + 1) * sizeof(posting));
    if (!ix->plist[t]) return ORC_E_NOMEM;
  }
  for (uint64_t d = 0; d < nlive; d++)
    for (uint64_t e = ix->dt_off[d]; e < ix->dt_off[d + 1]; e++) {
      uint32_t t = ix->dt_term[e];
      ix->plist[t][ix->plen[t]].doc = (uint32_t)d;
      ix->plist[t][ix->plen[t]].tf = ix->dt_tf[e];
      ix->plen[t]++;
    }
  ix->committed = 1;
  return ORC_OK;
}

uint64_t orc_num_docs(const orc_index *ix) { return ix->nlive; }
uint64_t orc_doc_count(const orc_index *ix) { return ix->doc_count; }
uint64_t orc_sum_ttf(const orc_index *ix) { return ix->sum_ttf; }
uint64_t orc_num_terms(const orc_index *ix) { return ix->terms.n; }
uint64_t orc_malformed_docs(const orc_index *ix, uint64_t *docs, uint64_t cap) {
  for (uint64_t i = 0; i < ix->n_malformed && i < cap; i++) docs[i] = ix->malformed[i];
  return ix->n_malformed;
}
uint32_t orc_doc_len(const orc_index *ix, uint64_t d) { return d < ix->nlive ? ix->doc_len[d] : 0; }
uint8_t orc_doc_norm(const orc_index *ix, uint64_t d) { return d < ix->nlive ? ix->doc_norm[d] : 0; }

uint64_t orc_doc_key(const orc_index *ix, uint64_t d, uint8_t *buf, uint64_t cap) {
  if (d >= ix->nlive) return 0;
  const stored_doc *sd = &ix->docs[ix->live[d]];
  memcpy(buf, sd->key, sd->key_len < cap ? sd->key_len : cap);
  return sd->key_len;
}

int64_t orc_doc_terms(const orc_index *ix, uint64_t d, char *buf, uint64_t buf_cap,
                      uint32_t *tfs, uint64_t cap) {
  if (d >= ix->nlive) return ORC_E_ARG;
  uint64_t a = ix->dt_off[d], z = ix->dt_off[d + 1], need = 0;
  for (uint64_t e = a; e < z; e++) need += ix->terms.len[ix->dt_term[e]] + 1;
  if (need > buf_cap || z - a > cap) return ORC_E_CAP;
  uint64_t p = 0;
  for (uint64_t e = a; e < z; e++) {
    uint32_t t = ix->dt_term[e];
    memcpy(buf + p, st_str(&ix->terms, t), ix->terms.len[t] + 1);
    p += ix->terms.len[t] + 1;
    tfs[e - a] = ix->dt_tf[e];
  }
  return (int64_t)(z - a);
}

int64_t orc_df(const orc_index *ix, const uint8_t *term, uint64_t len) {
  int64_t id = st_find(&ix->terms, term, len);
  return id < 0 ? 0 : (int64_t)ix->df[id];
}

int64_t orc_vocab(const orc_index *ix, char *buf, uint64_t buf_cap, uint32_t *df, uint64_t cap) {
  uint64_t V = ix->terms.n, need = 0;
  for (uint64_t t = 0; t < V; t++) need += ix->terms.len[t] + 1;
  if (need > buf_cap || V > cap) return ORC_E_CAP;
  memcpy(buf, ix->terms.arena, need);
  for (uint64_t t = 0; t < V; t++) df[t] = (uint32_t)ix->df[t];
  return (int64_t)V;
}

int orc_set_global_stats(orc_index *ix, uint64_t doc_count, uint64_t sum_ttf) {
  ix->g_doc_count = doc_count;
  ix->g_sum_ttf = sum_ttf;
  if (doc_count == 0) { st_free(&ix->g_terms); st_init(&ix->g_terms); }
  return ORC_OK;
}

int orc_set_global_df(orc_index *ix, const uint8_t *term, uint64_t len, uint64_t df) {
  int64_t id = st_insert(&ix->g_terms, term, len);
  if (id < 0) return ORC_E_NOMEM;
  if ((uint64_t)id >= ix->g_df_cap) {
    uint64_t nc = ix->g_df_cap ? ix->g_df_cap * 2 : 1024;
    while (nc <= (uint64_t)id) nc *= 2;
    uint64_t *g = (uint64_t *)realloc(ix->g_df, nc * sizeof(uint64_t));
    if (!g) return ORC_E_NOMEM;
    ix->g_df = g; ix->g_df_cap = nc;
  }
  ix->g_df[id] = df;
  return ORC_OK;
}

/* ------------------------------------------------------------------ */
/* Query: Worker.searchIndex (Worker.java:225-230) =
 *   new QueryParser("contents", new StandardAnalyzer()).parse(QueryParser.escape(q))
 *   searcher.search(query, Integer.MAX_VALUE)
 * restated from Lucene 9.8.0:
 *  - QueryParser.escape backslash-escapes  \ + - ! ( ) : ^ [ ] " { } ~ * ? | & /
 *    so the classic grammar (queryparser/classic/QueryParser.jj) only sees
 *    whitespace-separated TERM chunks and the operator words AND / OR / NOT:
 *      Query := Modifiers Clause (Conjunction Modifiers Clause)*
 *      Conjunction := [AND | OR], Modifiers := [NOT], Clause := TERM
 *    anything else (empty query, leading AND/OR, trailing or doubled
 *    operator) is a ParseException, which Worker turns into [] (:182-185);
 *  - QueryParserBase.addClause, default operator OR: AND marks the previous
 *    clause MUST unless it is MUST_NOT and the new clause MUST; NOT marks it
 *    MUST_NOT; else SHOULD.  A chunk the analyzer empties adds no clause;
 *  - QueryBuilder.createFieldQuery (not quoted, autoGeneratePhraseQueries
 *    false): one token -> TermQuery, several -> BooleanQuery of SHOULD
 *    TermQuerys (analyzeMultiBoolean);
 *  - BooleanQuery.Builder.add: more than IndexSearcher.maxClauseCount (1024)
 *    clauses in one node -> TooManyClauses (-> ParseException / exception);
 *  - BooleanQuery.rewrite to its fixpoint: nested clauses rewritten first
 *    (their duplicate SHOULD terms merged, a one-term result is
 *    BoostQuery(term, n)); duplicate SHOULD clauses and duplicate MUST
 *    clauses merged by summing their (unwrapped) boosts in double; nested
 *    pure disjunctions in SHOULD position flattened [verify: restated, no
 *    Lucene artefact in this image];
 *  - scoring (Boolean2ScorerSupplier): no MUST -> SHOULD disjunction
 *    (float)(double sum); MUST only -> conjunction (float)(double sum of the
 *    clause scores; a nested clause scores (float)(double sum of its terms));
 *    MUST + SHOULD -> ReqOptSumScorer: required float + optional float (float
 *    addition) when a SHOULD matches; MUST_NOT removes documents; no positive
 *    clause -> no hits.  TermQuery weight = boost * idf (BM25Scorer). */
#define OQ_SHOULD 0
#define OQ_MUST 1
#define OQ_MUST_NOT 2
#define OQ_MAX_CLAUSES 1024

/* classic QueryParser _WHITESPACE: " " | "\t" | "\n" | "\r" | "　"; length in bytes or 0 */
static int qp_ws(const uint8_t *q, uint64_t n, uint64_t i) {
  if (q[i] == ' ' || q[i] == '\t' || q[i] == '\n' || q[i] == '\r') return 1;
  if (q[i] == 0xE3 && i + 2 < n && q[i + 1] == 0x80 && q[i + 2] == 0x80) return 3;
  return 0;
}

typedef struct {
  int occur;
  uint32_t t0, nt;      /* distinct tokens: entries [t0, t0 + nt) of the token table */
  double boost;         /* clause boost after MUST de-duplication */
  int dead;             /* merged into an earlier identical clause */
} oq_clause;

typedef struct {
  strtab toks;                     /* distinct token strings of the whole query */
  uint32_t *tid; float *tcnt;      /* token table: token id + count inside its clause */
  uint32_t nt, tcap;
  oq_clause *cl; uint32_t ncl, clcap;
} oq_query;

static void oq_free(oq_query *Q) {
  st_free(&Q->toks); free(Q->tid); free(Q->tcnt); free(Q->cl);
}

static int oq_push_tok(oq_query *Q, uint32_t id) {
  if (Q->nt == Q->tcap) {
    uint32_t nc = Q->tcap ? Q->tcap * 2 : 64;
    uint32_t *a = (uint32_t *)realloc(Q->tid, nc * 4);
    if (!a) return ORC_E_NOMEM;
    Q->tid = a;
    float *c = (float *)realloc(Q->tcnt, nc * 4);
    if (!c) return ORC_E_NOMEM;
    Q->tcnt = c; Q->tcap = nc;
  }
  Q->tid[Q->nt] = id; Q->tcnt[Q->nt] = 1.0f; Q->nt++;
  return ORC_OK;
}

/* addClause for one TERM chunk [s, s + len) */
static int oq_add_clause(oq_query *Q, int conj_and, int mod_not, const uint8_t *s, uint64_t len) {
  if (Q->ncl > 0 && conj_and && Q->cl[Q->ncl - 1].occur != OQ_MUST_NOT) Q->cl[Q->ncl - 1].occur = OQ_MUST;
  uint64_t cap = len / 2 + 2;
  uint32_t *st = (uint32_t *)malloc(cap * 4), *ln = (uint32_t *)malloc(cap * 4);
  uint8_t lb[2048];
  if (!st || !ln) { free(st); free(ln); return ORC_E_NOMEM; }
  int64_t nt = orc_tokenize(s, len, 255, st, ln, cap);
  if (nt < 0) { free(st); free(ln); return ORC_E_UNSUPPORTED; }
  if (nt == 0) { free(st); free(ln); return ORC_OK; }
  if (nt > OQ_MAX_CLAUSES) { free(st); free(ln); return ORC_E_SYNTAX; }
  if (Q->ncl == Q->clcap) {
    uint32_t nc = Q->clcap ? Q->clcap * 2 : 16;
    oq_clause *c = (oq_clause *)realloc(Q->cl, nc * sizeof(oq_clause));
    if (!c) { free(st); free(ln); return ORC_E_NOMEM; }
    Q->cl = c; Q->clcap = nc;
  }
  oq_clause *c = &Q->cl[Q->ncl++];
  c->occur = mod_not ? OQ_MUST_NOT : (conj_and ? OQ_MUST : OQ_SHOULD);
  c->t0 = Q->nt; c->nt = 0; c->boost = 1.0; c->dead = 0;
  for (int64_t t = 0; t < nt; t++) {
    const uint64_t ll = orc_lower_utf8(s + st[t], ln[t], lb);
    int64_t id = st_insert(&Q->toks, lb, ll);
    if (id < 0) { free(st); free(ln); return ORC_E_NOMEM; }
    uint32_t k = c->t0;
    while (k < c->t0 + c->nt && Q->tid[k] != (uint32_t)id) k++;
    if (k < c->t0 + c->nt) { Q->tcnt[k] += 1.0f; continue; }   /* the nested query's SHOULD dedupe */
    if (oq_push_tok(Q, (uint32_t)id) != ORC_OK) { free(st); free(ln); return ORC_E_NOMEM; }
    c->nt++;
  }
  free(st); free(ln);
  return ORC_OK;
}

/* clause equality after rewrite: a one-token clause is its term (its count
 * is a BoostQuery boost, unwrapped by the dedupe); a nested clause equals a
 * nested clause with the same (token, count) multiset */
static int oq_same(const oq_query *Q, const oq_clause *a, const oq_clause *b) {
  if (a->nt != b->nt) return 0;
  if (a->nt == 1) return Q->tid[a->t0] == Q->tid[b->t0];
  for (uint32_t i = 0; i < a->nt; i++) {
    uint32_t j = 0;
    while (j < b->nt && Q->tid[b->t0 + j] != Q->tid[a->t0 + i]) j++;
    if (j == b->nt || Q->tcnt[b->t0 + j] != Q->tcnt[a->t0 + i]) return 0;
  }
  return 1;
}

static int oq_parse(const uint8_t *q, uint64_t n, oq_query *Q) {
  memset(Q, 0, sizeof *Q);
  if (st_init(&Q->toks) != ORC_OK) return ORC_E_NOMEM;
  /* lexer: whitespace-separated chunks, AND / OR / NOT exactly -> operators */
  enum { K_TERM, K_AND, K_OR, K_NOT };
  uint64_t m = 0, cap = 16;
  uint64_t *sa = (uint64_t *)malloc(cap * 8), *sl = (uint64_t *)malloc(cap * 8);
  int *kd = (int *)malloc(cap * sizeof(int));
  if (!sa || !sl || !kd) { free(sa); free(sl); free(kd); return ORC_E_NOMEM; }
  for (uint64_t i = 0; i < n;) {
    while (i < n && qp_ws(q, n, i)) i += (uint64_t)qp_ws(q, n, i);
    if (i >= n) break;
    uint64_t j = i;
    while (j < n && !qp_ws(q, n, j)) j++;
    if (m == cap) {
      cap *= 2;
      sa = (uint64_t *)realloc(sa, cap * 8); sl = (uint64_t *)realloc(sl, cap * 8);
      kd = (int *)realloc(kd, cap * sizeof(int));
      if (!sa || !sl || !kd) return ORC_E_NOMEM;
    }
    const uint64_t w = j - i;
    sa[m] = i; sl[m] = w;
    kd[m] = (w == 3 && !memcmp(q + i, "AND", 3)) ? K_AND
          : (w == 2 && !memcmp(q + i, "OR", 2)) ? K_OR
          : (w == 3 && !memcmp(q + i, "NOT", 3)) ? K_NOT : K_TERM;
    m++;
    i = j;
  }
  int rc = ORC_OK;
  uint64_t p = 0;
  int first = 1;
  while (rc == ORC_OK && (first || p < m)) {
    int conj_and = 0, mod_not = 0;
    if (!first && (kd[p] == K_AND || kd[p] == K_OR)) { conj_and = kd[p] == K_AND; p++; }
    if (p < m && kd[p] == K_NOT) { mod_not = 1; p++; }
    if (p >= m || kd[p] != K_TERM) { rc = ORC_E_SYNTAX; break; }
    rc = oq_add_clause(Q, conj_and, mod_not, q + sa[p], sl[p]);
    p++;
    first = 0;
  }
  free(sa); free(sl); free(kd);
  if (rc != ORC_OK) return rc;
  if (Q->ncl > OQ_MAX_CLAUSES) return ORC_E_SYNTAX;
  /* MUST de-duplication (boosts summed in double on the first occurrence) */
  for (uint32_t i = 0; i < Q->ncl; i++) {
    oq_clause *a = &Q->cl[i];
    if (a->occur != OQ_MUST || a->dead) continue;
    a->boost = a->nt == 1 ? (double)Q->tcnt[a->t0] : 1.0;
    for (uint32_t j = i + 1; j < Q->ncl; j++) {
      oq_clause *b = &Q->cl[j];
      if (b->occur == OQ_MUST && !b->dead && oq_same(Q, a, b)) {
        a->boost += b->nt == 1 ? (double)Q->tcnt[b->t0] : 1.0;
        b->dead = 1;
      }
    }
  }
  /* the flattening builder: every distinct SHOULD clause's terms + the other
   * distinct clauses must fit maxClauseCount */
  int nested = 0;
  uint64_t flat = 0;
  for (uint32_t i = 0; i < Q->ncl; i++) {
    const oq_clause *a = &Q->cl[i];
    if (a->dead) continue;
    int dup = 0;
    for (uint32_t j = 0; j < i && !dup; j++)
      dup = Q->cl[j].occur == a->occur && !Q->cl[j].dead && a->occur != OQ_MUST && oq_same(Q, &Q->cl[j], a);
    if (dup) continue;
    if (a->occur == OQ_SHOULD) { flat += a->nt; nested |= a->nt > 1; }
    else flat += 1;
  }
  if (nested && flat > OQ_MAX_CLAUSES) return ORC_E_SYNTAX;
  return ORC_OK;
}

/* SHOULD terms of the rewritten query: flattened, duplicates merged
 * (first appearance order), boost = summed count */
static uint32_t oq_should(const oq_query *Q, uint32_t *ids, double *boost) {
  uint32_t ns = 0;
  for (uint32_t i = 0; i < Q->ncl; i++) {
    const oq_clause *c = &Q->cl[i];
    if (c->occur != OQ_SHOULD) continue;
    for (uint32_t k = c->t0; k < c->t0 + c->nt; k++) {
      uint32_t j = 0;
      while (j < ns && ids[j] != Q->tid[k]) j++;
      if (j == ns) { ids[ns] = Q->tid[k]; boost[ns] = 0.0; ns++; }
      boost[j] += (double)Q->tcnt[k];
    }
  }
  return ns;
}

int64_t orc_query_terms(const uint8_t *q, uint64_t n, char *buf, uint64_t buf_cap,
                        float *boosts, uint64_t cap) {
  oq_query Q;
  int rc = oq_parse(q, n, &Q);
  if (rc != ORC_OK) { oq_free(&Q); return rc; }
  uint32_t *ids = (uint32_t *)malloc((Q.nt + 1) * 4);
  double *bs = (double *)malloc((Q.nt + 1) * 8);
  if (!ids || !bs) { free(ids); free(bs); oq_free(&Q); return ORC_E_NOMEM; }
  uint32_t ns = oq_should(&Q, ids, bs);
  uint64_t need = 0;
  for (uint32_t t = 0; t < ns; t++) need += Q.toks.len[ids[t]] + 1;
  int64_t ret = (int64_t)ns;
  if (need > buf_cap || ns > cap) ret = ORC_E_CAP;
  else {
    uint64_t off = 0;
    for (uint32_t t = 0; t < ns; t++) {
      memcpy(buf + off, st_str(&Q.toks, ids[t]), Q.toks.len[ids[t]] + 1);
      off += Q.toks.len[ids[t]] + 1;
      boosts[t] = (float)bs[t];
    }
  }
  free(ids); free(bs); oq_free(&Q);
  return ret;
}

typedef struct { float score; uint32_t doc; } hit;

static int hit_cmp(const void *a, const void *b) {
  const hit *x = (const hit *)a, *y = (const hit *)b;
  if (x->score != y->score) return x->score > y->score ? -1 : 1;
  return x->doc < y->doc ? -1 : (x->doc > y->doc);
}

/* BM25 weight of query token id under the statistics in force; returns the
 * index term id or -1 (absent: TermWeight.scorer == null) */
static int64_t oq_term(const orc_index *ix, const oq_query *Q, uint32_t id, uint64_t doc_count, float boost,
                       float *w) {
  const char *p = st_str(&Q->toks, id);
  const uint64_t len = Q->toks.len[id];
  int64_t t = st_find(&ix->terms, (const uint8_t *)p, len);
  if (t < 0 || doc_count == 0) return -1;
  uint64_t df = ix->df[t];
  if (ix->g_doc_count) {
    int64_t gid = st_find(&ix->g_terms, (const uint8_t *)p, len);
    df = gid >= 0 ? ix->g_df[gid] : df;
  }
  *w = boost * orc_idf(df, doc_count);
  return t;
}

int orc_search(const orc_index *ix, const uint8_t *q, uint64_t q_len, uint32_t k,
               uint32_t *docs, float *scores, uint64_t cap, uint64_t *n_out) {
  *n_out = 0;
  if (!ix->committed) return ORC_E_ARG;
  oq_query Q;
  int rc = oq_parse(q, q_len, &Q);
  if (rc != ORC_OK) { oq_free(&Q); return rc; }
  const uint64_t N = ix->nlive;
  const uint64_t doc_count = ix->g_doc_count ? ix->g_doc_count : ix->doc_count;
  const uint64_t sum_ttf = ix->g_doc_count ? ix->g_sum_ttf : ix->sum_ttf;
  float cache[256];
  if (doc_count > 0) orc_norm_cache(ix->k1, ix->b, orc_avgdl(sum_ttf, doc_count), cache);
  double *sacc = (double *)calloc(N + 1, sizeof(double));   /* SHOULD double sum */
  double *racc = (double *)calloc(N + 1, sizeof(double));   /* MUST: double sum of clause floats */
  double *cacc = (double *)calloc(N + 1, sizeof(double));   /* current MUST clause */
  uint8_t *smatch = (uint8_t *)calloc(N + 1, 1), *cmatch = (uint8_t *)calloc(N + 1, 1);
  uint8_t *excl = (uint8_t *)calloc(N + 1, 1);
  uint32_t *rcount = (uint32_t *)calloc(N + 1, 4);
  uint32_t *ids = (uint32_t *)malloc((Q.nt + 1) * 4);
  double *bs = (double *)malloc((Q.nt + 1) * 8);
  if (!sacc || !racc || !cacc || !smatch || !cmatch || !excl || !rcount || !ids || !bs) rc = ORC_E_NOMEM;
  uint32_t n_must = 0, ns = 0;
  if (rc == ORC_OK) {
    /* SHOULD (flattened, merged) */
    ns = oq_should(&Q, ids, bs);
    for (uint32_t s = 0; s < ns; s++) {
      float w;
      int64_t t = oq_term(ix, &Q, ids[s], doc_count, (float)bs[s], &w);
      if (t < 0) continue;
      for (uint64_t e = 0; e < ix->plen[t]; e++) {
        const posting *ps = &ix->plist[t][e];
        sacc[ps->doc] += (double)orc_bm25(w, ps->tf, cache[ix->doc_norm[ps->doc]]);
        smatch[ps->doc] = 1;
      }
    }
    /* MUST clauses, in order: clause score, then the conjunction's double sum */
    for (uint32_t c = 0; c < Q.ncl; c++) {
      const oq_clause *cl = &Q.cl[c];
      if (cl->occur != OQ_MUST || cl->dead) continue;
      n_must++;
      memset(cmatch, 0, N + 1);
      const float cb = (float)cl->boost;
      for (uint32_t i = cl->t0; i < cl->t0 + cl->nt; i++) {
        float tb = cl->nt == 1 ? cb : cb * Q.tcnt[i];
        float w;
        int64_t t = oq_term(ix, &Q, Q.tid[i], doc_count, tb, &w);
        if (t < 0) continue;
        for (uint64_t e = 0; e < ix->plen[t]; e++) {
          const posting *ps = &ix->plist[t][e];
          const double sc = (double)orc_bm25(w, ps->tf, cache[ix->doc_norm[ps->doc]]);
          cacc[ps->doc] = cmatch[ps->doc] ? cacc[ps->doc] + sc : sc;
          cmatch[ps->doc] = 1;
        }
      }
      for (uint64_t d = 0; d < N; d++)
        if (cmatch[d]) { racc[d] += (double)(float)cacc[d]; rcount[d]++; }
    }
    /* MUST_NOT */
    for (uint32_t c = 0; c < Q.ncl; c++) {
      const oq_clause *cl = &Q.cl[c];
      if (cl->occur != OQ_MUST_NOT) continue;
      for (uint32_t i = cl->t0; i < cl->t0 + cl->nt; i++) {
        float w;
        int64_t t = oq_term(ix, &Q, Q.tid[i], doc_count, 1.0f, &w);
        if (t < 0) continue;
        for (uint64_t e = 0; e < ix->plen[t]; e++) excl[ix->plist[t][e].doc] = 1;
      }
    }
  }
  hit *h = rc == ORC_OK ? (hit *)malloc((N + 1) * sizeof(hit)) : NULL;
  if (rc == ORC_OK && !h) rc = ORC_E_NOMEM;
  uint64_t nh = 0;
  if (rc == ORC_OK) {
    for (uint64_t d = 0; d < N; d++) {
      if (excl[d]) continue;
      float sc;
      if (n_must) {
        if (rcount[d] != n_must) continue;
        const float req = (float)racc[d];
        if (smatch[d]) { const float opt = (float)sacc[d]; sc = req + opt; }
        else sc = req;
      } else {
        if (!smatch[d]) continue;
        sc = (float)sacc[d];
      }
      h[nh].score = sc; h[nh].doc = (uint32_t)d; nh++;
    }
    qsort(h, nh, sizeof(hit), hit_cmp);
    uint64_t out = (k == 0 || k > nh) ? nh : k;
    *n_out = out;
    if (out > cap) rc = ORC_E_CAP;
    else
      for (uint64_t i = 0; i < out; i++) { docs[i] = h[i].doc; scores[i] = h[i].score; }
  }
  free(h); free(sacc); free(racc); free(cacc); free(smatch); free(cmatch); free(excl); free(rcount);
  free(ids); free(bs); oq_free(&Q);
  return rc;
}

/* ------------------------------------------------------------------ */
/* Leader.start merge (Leader.java:73-88): HashMap.merge(name, score,
 * Double::sum) in response order, then TreeMap<String, Double> order =
 * String.compareTo = lexicographic over UTF-16 code units.  Each name is
 * transcoded UTF-8 -> UTF-16 (surrogate pairs for code points >= 0x10000;
 * an invalid byte maps to the unit 0xFFFD + byte, keeping distinct names
 * distinct) and the unit arrays are compared. */
typedef struct { uint16_t *u; uint64_t n; } u16name;

static u16name to_utf16(const uint8_t *s, uint64_t n) {
  u16name r;
  r.u = (uint16_t *)malloc((2 * n + 1) * sizeof(uint16_t));
  r.n = 0;
  uint64_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    uint32_t len = c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : (c & 0xF8) == 0xF0 ? 4 : 0;
    uint32_t cp = 0, ok = len && i + len <= n;
    if (ok) {
      cp = len == 1 ? c : (uint32_t)(c & (0x7F >> len));
      for (uint32_t k = 1; k < len; k++) {
        if ((s[i + k] & 0xC0) != 0x80) { ok = 0; break; }
        cp = (cp << 6) | (s[i + k] & 0x3F);
      }
    }
    if (!ok) { r.u[r.n++] = 0xFFFD; r.u[r.n++] = c; i++; continue; }
    if (cp >= 0x10000) {
      cp -= 0x10000;
      r.u[r.n++] = (uint16_t)(0xD800 + (cp >> 10));
      r.u[r.n++] = (uint16_t)(0xDC00 + (cp & 0x3FF));
    } else {
      r.u[r.n++] = (uint16_t)cp;
    }
    i += len;
  }
  return r;
}

static int u16_cmp(const u16name *x, const u16name *y) {
  uint64_t m = x->n < y->n ? x->n : y->n;
  for (uint64_t i = 0; i < m; i++)
    if (x->u[i] != y->u[i]) return x->u[i] < y->u[i] ? -1 : 1;
  return x->n == y->n ? 0 : (x->n < y->n ? -1 : 1);
}

static const u16name *g_u16;
static int name_cmp_idx(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  int c = u16_cmp(&g_u16[x], &g_u16[y]);
  if (c) return c;
  return x < y ? -1 : (x > y);                   /* stable: first occurrence first */
}

int64_t orc_leader_merge(const uint8_t *names, const uint64_t *offsets, uint64_t n,
                         const double *scores, uint64_t *out_first, double *out_sum) {
  uint64_t *idx = (uint64_t *)malloc((n + 1) * sizeof(uint64_t));
  u16name *u = (u16name *)malloc((n + 1) * sizeof(u16name));
  if (!idx || !u) { free(idx); free(u); return ORC_E_NOMEM; }
  for (uint64_t i = 0; i < n; i++) {
    idx[i] = i;
    u[i] = to_utf16(names + offsets[i], offsets[i + 1] - offsets[i]);
  }
  g_u16 = u;
  qsort(idx, n, sizeof(uint64_t), name_cmp_idx);
  int64_t m = -1;
  uint64_t prev = 0;
  for (uint64_t r = 0; r < n; r++) {
    uint64_t i = idx[r];
    if (m < 0 || u16_cmp(&u[prev], &u[i]) != 0) { m++; out_first[m] = i; prev = i; }
  }
  /* Double::sum in response order (HashMap.merge is applied in list order) */
  for (uint64_t r = 0; r <= (uint64_t)m && m >= 0; r++) out_sum[r] = 0.0;
  for (uint64_t i = 0; i < n; i++) {
    int64_t lo = 0, hi = m;
    while (lo <= hi) {
      int64_t mid = (lo + hi) / 2;
      int c = u16_cmp(&u[out_first[mid]], &u[i]);
      if (c == 0) { out_sum[mid] += scores[i]; break; }
      if (c < 0) lo = mid + 1; else hi = mid - 1;
    }
  }
  for (uint64_t i = 0; i < n; i++) free(u[i].u);
  free(u); free(idx);
  return m + 1;
}

/* ---- CPU baseline: one index per thread (bench.py cpu_baseline) ---------- */
typedef struct {
  const uint8_t *text;
  const uint64_t *offsets;
  uint64_t lo, hi, ttf;
  int rc;
} bulk_part;

static void *bulk_worker(void *arg) {
  bulk_part *w = (bulk_part *)arg;
  orc_index *ix = orc_create(1.2f, 0.75f);
  if (!ix) { w->rc = ORC_E_NOMEM; return NULL; }
  char key[24];
  for (uint64_t d = w->lo; d < w->hi && w->rc == ORC_OK; d++) {
    const int kl = snprintf(key, sizeof key, "%llu", (unsigned long long)d);
    const int rc = orc_add_doc(ix, (const uint8_t *)key, (uint64_t)kl, w->text + w->offsets[d],
                               w->offsets[d + 1] - w->offsets[d]);
    if (rc != ORC_OK && rc != ORC_E_UNSUPPORTED) w->rc = rc;
  }
  if (w->rc == ORC_OK) w->rc = orc_commit(ix);
  w->ttf = orc_sum_ttf(ix);
  orc_destroy(ix);
  return NULL;
}

int orc_bulk_build(const uint8_t *text, const uint64_t *offsets, uint64_t n_docs, uint32_t n_threads,
                   double *seconds, uint64_t *sum_ttf) {
  if (!text || !offsets || !seconds || !sum_ttf || n_threads == 0) return ORC_E_ARG;
  bulk_part *parts = (bulk_part *)calloc(n_threads, sizeof(bulk_part));
  pthread_t *th = (pthread_t *)calloc(n_threads, sizeof(pthread_t));
  if (!parts || !th) { free(parts); free(th); return ORC_E_NOMEM; }
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  uint32_t started = 0;
  int rc = ORC_OK;
  for (uint32_t t = 0; t < n_threads; t++) {
    parts[t] = (bulk_part){text, offsets, n_docs * t / n_threads, n_docs * (t + 1) / n_threads, 0, ORC_OK};
    if (pthread_create(&th[t], NULL, bulk_worker, &parts[t]) != 0) { rc = ORC_E_NOMEM; break; }
    started++;
  }
  uint64_t ttf = 0;
  for (uint32_t t = 0; t < started; t++) {
    pthread_join(th[t], NULL);
    if (parts[t].rc != ORC_OK) rc = parts[t].rc;
    ttf += parts[t].ttf;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  *seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  *sum_ttf = ttf;
  free(parts);
  free(th);
  return rc;
}
