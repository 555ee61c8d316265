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
#include "tfidf_oracle.h"

#include <math.h>
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
  free(ix->live); free(ix->doc_len); free(ix->doc_norm);
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

/* qsort_r is a GNU extension; keep a small insertion+merge sort instead. */
static void sort_terms(uint32_t *ids, uint32_t *tfs, uint64_t n, const strtab *t) {
  for (uint64_t i = 1; i < n; i++) {
    uint32_t a = ids[i], f = tfs[i];
    uint64_t j = i;
    while (j > 0 && cmp_term_ids(&ids[j - 1], &a, (void *)t) > 0) {
      ids[j] = ids[j - 1]; tfs[j] = tfs[j - 1]; j--;
    }
    ids[j] = a; tfs[j] = f;
  }
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
/* Query analysis: QueryParser.escape + classic QueryParser (default OR,
 * splitOnWhitespace) + StandardAnalyzer per chunk.  escape() neutralises
 * every special character except the operator WORDS AND/OR/NOT, which stay
 * operators; those are reported as ORC_E_UNSUPPORTED.  With only escaped
 * characters, the parse is the multiset of analysed tokens (whitespace is a
 * break character for the analyzer as well), de-duplicated by
 * BooleanQuery.rewrite with boost = occurrence count. */
/* classic QueryParser _WHITESPACE: " " | "\t" | "\n" | "\r" | "\u3000"; length in bytes or 0 */
static int qp_ws(const uint8_t *q, uint64_t n, uint64_t i) {
  if (q[i] == ' ' || q[i] == '\t' || q[i] == '\n' || q[i] == '\r') return 1;
  if (q[i] == 0xE3 && i + 2 < n && q[i + 1] == 0x80 && q[i + 2] == 0x80) return 3;
  return 0;
}

int64_t orc_query_terms(const uint8_t *q, uint64_t n, char *buf, uint64_t buf_cap,
                        float *boosts, uint64_t cap) {
  /* operator words */
  uint64_t i = 0;
  while (i < n) {
    while (i < n && qp_ws(q, n, i)) i += (uint64_t)qp_ws(q, n, i);
    uint64_t j = i;
    while (j < n && !qp_ws(q, n, j)) j++;
    uint64_t w = j - i;
    if ((w == 3 && (memcmp(q + i, "AND", 3) == 0 || memcmp(q + i, "NOT", 3) == 0)) ||
        (w == 2 && memcmp(q + i, "OR", 2) == 0))
      return ORC_E_UNSUPPORTED;
    i = j;
  }
  uint64_t tok_cap = n / 2 + 2;
  uint32_t *st = (uint32_t *)malloc(tok_cap * 4), *ln = (uint32_t *)malloc(tok_cap * 4);
  if (!st || !ln) return ORC_E_NOMEM;
  /* analyse chunk by chunk (restart context at each chunk, as QueryParser does) */
  strtab qt; st_init(&qt);
  float *cnt = (float *)calloc(tok_cap + 1, sizeof(float));
  uint8_t lb[2048];
  i = 0;
  while (i < n) {
    while (i < n && qp_ws(q, n, i)) i += (uint64_t)qp_ws(q, n, i);
    uint64_t j = i;
    while (j < n && !qp_ws(q, n, j)) j++;
    int64_t nt = orc_tokenize(q + i, j - i, 255, st, ln, tok_cap);
    if (nt < 0) { st_free(&qt); free(cnt); free(st); free(ln); return nt; }
    for (int64_t t = 0; t < nt; t++) {
      const uint64_t ll = orc_lower_utf8(q + i + st[t], ln[t], lb);
      int64_t id = st_insert(&qt, lb, ll);
      cnt[id] += 1.0f;
    }
    i = j;
  }
  uint64_t need = 0;
  for (uint64_t t = 0; t < qt.n; t++) need += qt.len[t] + 1;
  int64_t ret = (int64_t)qt.n;
  if (need > buf_cap || qt.n > cap) ret = ORC_E_CAP;
  else {
    memcpy(buf, qt.arena, need);
    for (uint64_t t = 0; t < qt.n; t++) boosts[t] = cnt[t];
  }
  st_free(&qt); free(cnt); free(st); free(ln);
  return ret;
}

typedef struct { float score; uint32_t doc; } hit;

static int hit_cmp(const void *a, const void *b) {
  const hit *x = (const hit *)a, *y = (const hit *)b;
  if (x->score != y->score) return x->score > y->score ? -1 : 1;
  return x->doc < y->doc ? -1 : (x->doc > y->doc);
}

int orc_search(const orc_index *ix, const uint8_t *q, uint64_t q_len, uint32_t k,
               uint32_t *docs, float *scores, uint64_t cap, uint64_t *n_out) {
  *n_out = 0;
  if (!ix->committed) return ORC_E_ARG;
  uint64_t tcap = q_len / 2 + 2;
  char *tb = (char *)malloc(q_len + tcap + 16);
  float *boost = (float *)malloc(tcap * sizeof(float));
  int64_t nq = orc_query_terms(q, q_len, tb, q_len + tcap + 16, boost, tcap);
  if (nq < 0) { free(tb); free(boost); return (int)nq; }
  uint64_t N = ix->nlive;
  uint64_t doc_count = ix->g_doc_count ? ix->g_doc_count : ix->doc_count;
  uint64_t sum_ttf = ix->g_doc_count ? ix->g_sum_ttf : ix->sum_ttf;
  double *acc = (double *)calloc(N + 1, sizeof(double));
  uint8_t *hitm = (uint8_t *)calloc(N + 1, 1);
  float cache[256];
  if (doc_count > 0) orc_norm_cache(ix->k1, ix->b, orc_avgdl(sum_ttf, doc_count), cache);
  const char *p = tb;
  for (int64_t t = 0; t < nq; t++) {
    uint64_t len = strlen(p);
    int64_t id = st_find(&ix->terms, (const uint8_t *)p, len);
    if (id >= 0 && doc_count > 0) {
      uint64_t df = ix->df[id];
      if (ix->g_doc_count) {
        int64_t gid = st_find(&ix->g_terms, (const uint8_t *)p, len);
        df = gid >= 0 ? ix->g_df[gid] : df;
      }
      float w = boost[t] * orc_idf(df, doc_count);
      for (uint64_t e = 0; e < ix->plen[id]; e++) {
        const posting *ps = &ix->plist[id][e];
        acc[ps->doc] += (double)orc_bm25(w, ps->tf, cache[ix->doc_norm[ps->doc]]);
        hitm[ps->doc] = 1;
      }
    }
    p += len + 1;
  }
  uint64_t nh = 0;
  for (uint64_t d = 0; d < N; d++) nh += hitm[d];
  hit *h = (hit *)malloc((nh + 1) * sizeof(hit));
  uint64_t j = 0;
  for (uint64_t d = 0; d < N; d++)
    if (hitm[d]) { h[j].score = (float)acc[d]; h[j].doc = (uint32_t)d; j++; }
  qsort(h, nh, sizeof(hit), hit_cmp);
  uint64_t out = (k == 0 || k > nh) ? nh : k;
  int rc = ORC_OK;
  *n_out = out;
  if (out > cap) rc = ORC_E_CAP;
  else
    for (uint64_t i = 0; i < out; i++) { docs[i] = h[i].doc; scores[i] = h[i].score; }
  free(h); free(acc); free(hitm); free(tb); free(boost);
  return rc;
}

/* ------------------------------------------------------------------ */
static const uint8_t *g_names;
static const uint64_t *g_offs;
static int name_cmp_idx(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  uint64_t lx = g_offs[x + 1] - g_offs[x], ly = g_offs[y + 1] - g_offs[y];
  uint64_t m = lx < ly ? lx : ly;
  int c = memcmp(g_names + g_offs[x], g_names + g_offs[y], m);
  if (c) return c;
  if (lx != ly) return lx < ly ? -1 : 1;
  return x < y ? -1 : (x > y);                   /* stable: first occurrence first */
}

int64_t orc_leader_merge(const uint8_t *names, const uint64_t *offsets, uint64_t n,
                         const double *scores, uint64_t *out_first, double *out_sum) {
  uint64_t *idx = (uint64_t *)malloc((n + 1) * sizeof(uint64_t));
  if (!idx) return ORC_E_NOMEM;
  for (uint64_t i = 0; i < n; i++) idx[i] = i;
  g_names = names; g_offs = offsets;
  qsort(idx, n, sizeof(uint64_t), name_cmp_idx);
  int64_t m = -1;
  uint64_t prev = 0;
  for (uint64_t r = 0; r < n; r++) {
    uint64_t i = idx[r];
    int same = 0;
    if (m >= 0) {
      uint64_t lp = offsets[prev + 1] - offsets[prev], li = offsets[i + 1] - offsets[i];
      same = lp == li && memcmp(names + offsets[prev], names + offsets[i], li) == 0;
    }
    if (!same) { m++; out_first[m] = i; out_sum[m] = 0.0; prev = i; }
  }
  /* Double::sum in response order (HashMap.merge is applied in list order) */
  for (uint64_t r = 0; r <= (uint64_t)m && m >= 0; r++) out_sum[r] = 0.0;
  for (uint64_t i = 0; i < n; i++) {
    /* binary search distinct index for name i */
    int64_t lo = 0, hi = m;
    while (lo <= hi) {
      int64_t mid = (lo + hi) / 2;
      uint64_t f = out_first[mid];
      uint64_t lf = offsets[f + 1] - offsets[f], li = offsets[i + 1] - offsets[i];
      uint64_t mm = lf < li ? lf : li;
      int c = memcmp(names + offsets[f], names + offsets[i], mm);
      if (!c) c = lf == li ? 0 : (lf < li ? -1 : 1);
      if (c == 0) { out_sum[mid] += scores[i]; break; }
      if (c < 0) lo = mid + 1; else hi = mid - 1;
    }
  }
  free(idx);
  return m + 1;
}
