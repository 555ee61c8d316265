// unicode_scan.h — the general (full-Unicode) StandardTokenizer scanner,
// shared by the device (k_tokenize_long's general phase) and the host (query
// analysis, tfidf_analyze).
//
// Restates Lucene 9.8.0 StandardTokenizerImpl (JFlex, `%unicode 9.0`) as
// called through StandardAnalyzer at Worker.java:71 (indexing) and :225
// (queries), followed by LowerCaseFilter (Character.toLowerCase per code point,
// JDK 17 of the reference's Dockerfile:1).  The JFlex grammar, per rule:
//
//   WORD    ENL* core (ENL+ core)* ENL*         core = KATAKANA (ENL* KATAKANA)*
//                                                     | (HgrpEx | NgrpEx | AgrpEx)+
//           Hgrp = HEBREW (SQUOTE | DQUOTE HEBREW)
//           Ngrp = NUMERIC ((ENL* | MidNum') NUMERIC)*      MidNum'    = MIDNUM | MIDNUMLET | SQUOTE
//           Agrp = AHL ((ENL* | MidLetter') AHL)*           MidLetter' = MIDLETTER | MIDNUMLET | SQUOTE
//           (AHL = ALETTER | HEBREW; NUMERIC covers the NUMERIC rule's extents)
//   SEA     ComplexContext+                    (Line_Break = SA runs: Thai, Lao, Khmer, Myanmar)
//   IDEO    one Han char;  HIRAGANA: one Hiragana char
//   EMOJI   pictographic char, then (ZWJ pictographic)*; a Regional_Indicator pair
//   skip    any other char ([^]), one at a time
//
// where every class X stands for X (Extend | Format | ZWJ)* (UAX#29 WB4): a
// "unit" below is a head char plus its trailing extenders.  The scanner is a
// longest-match DFA over units (states kW*); tokens longer than 255 UTF-16
// units are cut at 255 and scanning restarts at the cut (the chop of the
// ASCII path, analysis.h / kernels_index.hip).
//
// Byte-level parallelism: no token contains an ASCII char of class OTHER
// (space, newline, most punctuation), and JFlex never looks behind, so the
// scan state just after such a byte is the start state.  The device splits a
// document at those bytes and scans the pieces independently (uc_split_byte).
#pragma once

#include <stdint.h>

#include "tfidf_common.h"
#include "unicode_tables.h"

namespace tfidf {

enum : uint32_t {
  kUcOther = 0, kUcALetter, kUcHebrew, kUcNumeric, kUcKatakana, kUcExtNumLet, kUcMidLetter, kUcMidNumLet,
  kUcMidNum, kUcSQuote, kUcDQuote, kUcExtend, kUcExtendSA, kUcZWJ, kUcSA, kUcHan, kUcHiragana, kUcRI, kUcEmoji
};

#if defined(__HIP_DEVICE_COMPILE__)
static __device__ const uint16_t kUcClassIndex[TFIDF_UC_CLASS_INDEX_N] = TFIDF_UC_CLASS_INDEX;
static __device__ const uint8_t kUcClassData[TFIDF_UC_CLASS_DATA_N] = TFIDF_UC_CLASS_DATA;
static __device__ const uint16_t kUcLowerIndex[TFIDF_UC_LOWER_INDEX_N] = TFIDF_UC_LOWER_INDEX;
static __device__ const int32_t kUcLowerData[TFIDF_UC_LOWER_DATA_N] = TFIDF_UC_LOWER_DATA;
#else
static const uint16_t kUcClassIndex[TFIDF_UC_CLASS_INDEX_N] = TFIDF_UC_CLASS_INDEX;
static const uint8_t kUcClassData[TFIDF_UC_CLASS_DATA_N] = TFIDF_UC_CLASS_DATA;
static const uint16_t kUcLowerIndex[TFIDF_UC_LOWER_INDEX_N] = TFIDF_UC_LOWER_INDEX;
static const int32_t kUcLowerData[TFIDF_UC_LOWER_DATA_N] = TFIDF_UC_LOWER_DATA;
#endif

constexpr uint32_t kUcBad = 0xFFFFFFFFu;

TFIDF_HD uint32_t uc_class(uint32_t cp) {
  return cp < 0x110000u ? kUcClassData[(uint32_t)kUcClassIndex[cp >> 8] * 256u + (cp & 255u)] : kUcOther;
}
TFIDF_HD uint32_t uc_lower(uint32_t cp) {
  return (uint32_t)((int32_t)cp + kUcLowerData[(uint32_t)kUcLowerIndex[cp >> 8] * 256u + (cp & 255u)]);
}
// ASCII classes without a table read (the generated table agrees: every
// ASCII class lookup of the host scanner goes through this function).
TFIDF_HD uint32_t uc_ascii_class(uint32_t c) {
  if ((c | 0x20u) - 'a' < 26u) return kUcALetter;
  if (c - '0' < 10u) return kUcNumeric;
  switch (c) {
    case '_': return kUcExtNumLet;
    case ':': return kUcMidLetter;
    case '.': return kUcMidNumLet;
    case ',': case ';': return kUcMidNum;
    case '\'': return kUcSQuote;
    case '"': return kUcDQuote;
    default: return kUcOther;
  }
}
TFIDF_HD bool uc_is_extender(uint32_t c) { return c == kUcExtend || c == kUcExtendSA || c == kUcZWJ; }
// ASCII byte after which the scan state is the start state (see header).
TFIDF_HD bool uc_split_byte(uint8_t b) { return b < 0x80 && uc_ascii_class(b) == kUcOther; }

// Strict UTF-8 (what Files.readString's decoder accepts, Worker.java:198):
// code point at byte i, *len bytes; kUcBad for a malformed, overlong,
// surrogate or truncated sequence.
TFIDF_HD uint32_t utf8_decode(const uint8_t *s, uint64_t n, uint64_t i, uint32_t *len) {
  const uint32_t b0 = s[i];
  if (b0 < 0x80u) { *len = 1; return b0; }
  auto cont = [&](uint64_t k, uint32_t lo, uint32_t hi) -> int32_t {
    if (i + k >= n) return -1;
    const uint32_t b = s[i + k];
    return (b >= lo && b <= hi) ? (int32_t)(b & 0x3Fu) : -1;
  };
  if (b0 < 0xC2u) return kUcBad;
  if (b0 < 0xE0u) {
    const int32_t c1 = cont(1, 0x80, 0xBF);
    if (c1 < 0) return kUcBad;
    *len = 2;
    return ((b0 & 0x1Fu) << 6) | (uint32_t)c1;
  }
  if (b0 < 0xF0u) {
    const int32_t c1 = cont(1, b0 == 0xE0u ? 0xA0 : 0x80, b0 == 0xEDu ? 0x9F : 0xBF), c2 = cont(2, 0x80, 0xBF);
    if (c1 < 0 || c2 < 0) return kUcBad;
    *len = 3;
    return ((b0 & 0x0Fu) << 12) | ((uint32_t)c1 << 6) | (uint32_t)c2;
  }
  if (b0 < 0xF5u) {
    const int32_t c1 = cont(1, b0 == 0xF0u ? 0x90 : 0x80, b0 == 0xF4u ? 0x8F : 0xBF), c2 = cont(2, 0x80, 0xBF),
                  c3 = cont(3, 0x80, 0xBF);
    if (c1 < 0 || c2 < 0 || c3 < 0) return kUcBad;
    *len = 4;
    return ((b0 & 0x07u) << 18) | ((uint32_t)c1 << 12) | ((uint32_t)c2 << 6) | (uint32_t)c3;
  }
  return kUcBad;
}

// Class source of the scanner: class of the char starting at byte i and its
// byte length, kUcBad for malformed UTF-8.  This one decodes and reads the
// tables (host; device fallback); the Unicode wave kernel reads classes
// precomputed in LDS instead (kernels_unicode.hip).
struct UcDecodeSrc {
  const uint8_t *s;
  uint64_t n;
  TFIDF_HD uint32_t at(uint64_t i, uint32_t *len) const {
    const uint32_t b = s[i];
    if (b < 0x80u) { *len = 1; return uc_ascii_class(b); }
    const uint32_t cp = utf8_decode(s, n, i, len);
    return cp == kUcBad ? kUcBad : uc_class(cp);
  }
};

// WORD rule DFA states (accepting: A, H, N, K, EAFTER, HSQ).
enum : uint32_t { kWStart = 0, kWELead, kWA, kWH, kWN, kWK, kWEAfter, kWHSq, kWHDq, kWAMid, kWNMid, kWDead };

TFIDF_HD bool uc_word_accepting(uint32_t st) { return st >= kWA && st <= kWHSq; }

TFIDF_HD uint32_t uc_word_next(uint32_t st, uint32_t c) {
  // successors common to every state that may start / continue a letter group
  switch (st) {
    case kWStart:
    case kWELead:
    case kWEAfter:
      if (c == kUcExtNumLet) return st == kWEAfter ? kWEAfter : kWELead;
      if (c == kUcALetter) return kWA;
      if (c == kUcHebrew) return kWH;
      if (c == kUcNumeric) return kWN;
      if (c == kUcKatakana) return kWK;
      return kWDead;
    case kWA:
    case kWH:
    case kWHSq:
      if (c == kUcALetter) return kWA;
      if (c == kUcHebrew) return kWH;
      if (c == kUcNumeric) return kWN;
      if (c == kUcExtNumLet) return kWEAfter;
      if (st == kWHSq) return kWDead;
      if (st == kWH && c == kUcSQuote) return kWHSq;
      if (st == kWH && c == kUcDQuote) return kWHDq;
      if (c == kUcMidLetter || c == kUcMidNumLet || c == kUcSQuote) return kWAMid;
      return kWDead;
    case kWN:
      if (c == kUcNumeric) return kWN;
      if (c == kUcALetter) return kWA;
      if (c == kUcHebrew) return kWH;
      if (c == kUcExtNumLet) return kWEAfter;
      if (c == kUcMidNum || c == kUcMidNumLet || c == kUcSQuote) return kWNMid;
      return kWDead;
    case kWK:
      if (c == kUcKatakana) return kWK;
      if (c == kUcExtNumLet) return kWEAfter;
      return kWDead;
    case kWHDq:
      return c == kUcHebrew ? kWH : kWDead;
    case kWAMid:
      if (c == kUcALetter) return kWA;
      if (c == kUcHebrew) return kWH;
      return kWDead;
    case kWNMid:
      return c == kUcNumeric ? kWN : kWDead;
    default:
      return kWDead;
  }
}

// One unit (head + extenders) starting at byte i: returns the head class and
// the byte after the unit in *end; *zwj_last = the unit ends with a ZWJ.
template <class Src>
TFIDF_HD uint32_t uc_unit(const Src &src, uint64_t n, uint64_t i, uint64_t *end, bool *zwj_last, bool *bad) {
  uint32_t l;
  const uint32_t c = src.at(i, &l);
  if (c == kUcBad) { *bad = true; *end = n; return kUcOther; }
  uint64_t p = i + l;
  bool z = false;
  while (p < n) {
    const uint32_t c2 = src.at(p, &l);
    if (c2 == kUcBad) { *bad = true; *end = n; return kUcOther; }
    if (!uc_is_extender(c2)) break;
    z = c2 == kUcZWJ;
    p += l;
  }
  *end = p;
  *zwj_last = z;
  return c;
}

// Next token starting in [*pos, stop) (a scan position); its extent is
// [*ts, *te) (not yet chopped).  Returns false when none is left or the text
// is malformed (*bad).  *pos is advanced past the token / skipped chars.
template <class Src>
TFIDF_HD bool uc_next_span(const Src &src, uint64_t n, uint64_t *pos, uint64_t stop, uint64_t *ts, uint64_t *te,
                           bool *bad) {
  while (*pos < stop && !*bad) {
    const uint64_t i = *pos;
    uint32_t l;
    const uint32_t c = src.at(i, &l);
    if (c == kUcBad) { *bad = true; return false; }
    if (c == kUcALetter || c == kUcHebrew || c == kUcNumeric || c == kUcKatakana || c == kUcExtNumLet) {
      uint32_t st = kWStart;
      uint64_t p = i, last = i, erun = i;
      while (p < n) {
        uint64_t e;
        bool z;
        const uint32_t uc = uc_unit(src, n, p, &e, &z, bad);
        if (*bad) return false;
        const uint32_t ns = uc_word_next(st, uc);
        if (ns == kWDead) break;
        st = ns;
        p = e;
        if (uc_word_accepting(st)) last = p;
        else if (st == kWELead) erun = p;
      }
      if (last > i) { *ts = i; *te = last; *pos = last; return true; }
      // An ENL run followed by no core: none of its suffixes matches either,
      // so JFlex skips it char by char — and an SA mark among its extenders
      // starts an SA run there.
      uint64_t q = i + l;
      while (q < erun) {
        if (src.at(q, &l) == kUcExtendSA) break;
        q += l;
      }
      *pos = q;
      continue;
    }
    if (c == kUcSA || c == kUcExtendSA) {            // SEA: run of Complex_Context chars (+ extenders)
      uint64_t p = i + l;
      while (p < n) {
        const uint32_t c2 = src.at(p, &l);
        if (c2 == kUcBad) { *bad = true; return false; }
        if (c2 != kUcSA && !uc_is_extender(c2)) break;
        p += l;
      }
      *ts = i; *te = p; *pos = p;
      return true;
    }
    if (c == kUcHan || c == kUcHiragana || c == kUcEmoji || c == kUcRI) {
      uint64_t e;
      bool z;
      uc_unit(src, n, i, &e, &z, bad);
      if (*bad) return false;
      if (c == kUcEmoji) {                           // ZWJ sequences
        while (z && e < n) {
          uint64_t e2;
          bool z2;
          const uint32_t c2 = uc_unit(src, n, e, &e2, &z2, bad);
          if (*bad) return false;
          if (c2 != kUcEmoji) break;
          e = e2;
          z = z2;
        }
      } else if (c == kUcRI) {                       // flag = Regional_Indicator pair
        uint64_t e2 = e;
        bool z2;
        const uint32_t c2 = e < n ? uc_unit(src, n, e, &e2, &z2, bad) : kUcOther;
        if (*bad) return false;
        if (c2 != kUcRI) { *pos = i + l; continue; }
        e = e2;
      }
      *ts = i; *te = e; *pos = e;
      return true;
    }
    *pos = i + l;                                    // [^]: skip one char
  }
  return false;
}

// Term bytes of the token [ts, te) into sink.push(byte): lower-cased code
// points, UTF-8, cut at 255 UTF-16 units (a supplementary char that would
// straddle the cut is left to the next token).  Returns the byte end consumed.
template <class Sink>
TFIDF_HD uint64_t uc_token_bytes(const uint8_t *s, uint64_t n, uint64_t ts, uint64_t te, Sink &kb) {
  uint32_t u16 = 0;
  uint64_t p = ts;
  while (p < te) {
    uint32_t l;
    const uint32_t cp = utf8_decode(s, n, p, &l);
    const uint32_t w = cp >= 0x10000u ? 2u : 1u;
    if (u16 + w > kMaxTokenLen) break;
    u16 += w;
    const uint32_t lc = cp < 0x80u ? (uint32_t)ascii_lower((uint8_t)cp) : uc_lower(cp);
    if (lc < 0x80u) {
      kb.push((uint8_t)lc);
    } else if (lc < 0x800u) {
      kb.push((uint8_t)(0xC0u | (lc >> 6)));
      kb.push((uint8_t)(0x80u | (lc & 0x3Fu)));
    } else if (lc < 0x10000u) {
      kb.push((uint8_t)(0xE0u | (lc >> 12)));
      kb.push((uint8_t)(0x80u | ((lc >> 6) & 0x3Fu)));
      kb.push((uint8_t)(0x80u | (lc & 0x3Fu)));
    } else {
      kb.push((uint8_t)(0xF0u | (lc >> 18)));
      kb.push((uint8_t)(0x80u | ((lc >> 12) & 0x3Fu)));
      kb.push((uint8_t)(0x80u | ((lc >> 6) & 0x3Fu)));
      kb.push((uint8_t)(0x80u | (lc & 0x3Fu)));
    }
    p += l;
  }
  return p;
}

TFIDF_HD uint64_t uc_token_key(const uint8_t *s, uint64_t n, uint64_t ts, uint64_t te, uint64_t *lo, uint64_t *hi,
                               uint64_t seed = 0) {
  KeyBuilder kb;
  const uint64_t p = uc_token_bytes(s, n, ts, te, kb);
  kb.finish(lo, hi, seed);
  return p;
}

// Are the tokens s1[0, n1) and s2[0, n2) (raw bytes, already cut at 255
// units) the same term, i.e. equal lower-cased code points?  Raw equality
// first (the common case: the same spelling).
TFIDF_HD bool uc_same_term(const uint8_t *s1, uint32_t n1, const uint8_t *s2, uint32_t n2) {
  if (n1 == n2) {
    uint32_t i = 0;
    while (i < n1 && s1[i] == s2[i]) i++;
    if (i == n1) return true;
  }
  uint64_t p1 = 0, p2 = 0;
  while (p1 < n1 && p2 < n2) {
    uint32_t l1, l2;
    const uint32_t c1 = utf8_decode(s1, n1, p1, &l1), c2 = utf8_decode(s2, n2, p2, &l2);
    if (c1 == kUcBad || c2 == kUcBad) return false;
    const uint32_t x1 = c1 < 0x80u ? (uint32_t)ascii_lower((uint8_t)c1) : uc_lower(c1);
    const uint32_t x2 = c2 < 0x80u ? (uint32_t)ascii_lower((uint8_t)c2) : uc_lower(c2);
    if (x1 != x2) return false;
    p1 += l1;
    p2 += l2;
  }
  return p1 == n1 && p2 == n2;
}

// Host/device loop body: next token in [*pos, stop) with its key; handles the
// 255-unit cut (scanning restarts at the cut).
template <class Src>
TFIDF_HD bool uc_next_token(const Src &src, const uint8_t *s, uint64_t n, uint64_t *pos, uint64_t stop, uint64_t *ts,
                            uint64_t *te, uint64_t *lo, uint64_t *hi, bool *bad, uint64_t seed = 0) {
  if (!uc_next_span(src, n, pos, stop, ts, te, bad)) return false;
  const uint64_t cut = uc_token_key(s, n, *ts, *te, lo, hi, seed);
  if (cut < *te) { *te = cut; *pos = cut; }
  return true;
}

TFIDF_HD bool uc_next_token(const uint8_t *s, uint64_t n, uint64_t *pos, uint64_t stop, uint64_t *ts, uint64_t *te,
                            uint64_t *lo, uint64_t *hi, bool *bad, uint64_t seed = 0) {
  return uc_next_token(UcDecodeSrc{s, n}, s, n, pos, stop, ts, te, lo, hi, bad, seed);
}

}  // namespace tfidf
