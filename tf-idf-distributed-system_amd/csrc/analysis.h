// analysis.h — host-side query analysis for tfidf_search (Worker.java:225-227:
// QueryParser("contents", new StandardAnalyzer()).parse(QueryParser.escape(q))).
//
// QueryParser.escape backslash-escapes every query-syntax character
// (\ + - ! ( ) : ^ [ ] " { } ~ * ? | & /), so the parse of an escaped string is
// a flat OR of per-chunk analysed tokens — except for the operator WORDS
// AND / OR / NOT, which escape() leaves alone.  Those are rejected
// (TFIDF_E_UNSUPPORTED_QUERY) rather than silently mis-scored.  Chunks are
// split on the classic QueryParser's whitespace (space, \t, \n, \r);
// BooleanQuery.rewrite de-duplicates SHOULD clauses with boost = count.
#pragma once

#include <stdint.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "tfidf_common.h"

namespace tfidf {

struct QueryTerm {
  std::string term;   // lower-cased analysed token
  float boost;        // occurrence count
};

// StandardTokenizer (ASCII UAX#29) over [s, s + n), tokens chopped at 255 with
// scanning restarted at the cut.  Emits lower-cased token strings.
inline void analyze_ascii(const uint8_t *s, uint64_t n, std::vector<std::string> *out) {
  auto cls = [&](uint64_t i) -> uint8_t { return wb_class(s[i]); };
  uint64_t lo = 0, i = 0;
  auto is_word = [&](uint64_t k) -> bool {
    uint8_t p = (k > lo) ? cls(k - 1) : 0;
    uint8_t x = (k + 1 < n) ? cls(k + 1) : 0;
    return wb_is_word(p, cls(k), x);
  };
  while (i < n) {
    if (!is_word(i)) { i++; continue; }
    uint64_t j = i;
    bool has_ld = false;
    while (j < n && is_word(j)) { has_ld |= (cls(j) & (kClsL | kClsD)) != 0; j++; }
    if (!has_ld) { i = j; continue; }
    uint64_t len = j - i;
    if (len > kMaxTokenLen) len = kMaxTokenLen;
    std::string t(len, '\0');
    for (uint64_t c = 0; c < len; c++) t[c] = (char)ascii_lower(s[i + c]);
    out->push_back(std::move(t));
    if (j - i > kMaxTokenLen) { lo = i + kMaxTokenLen; i = lo; continue; }
    i = j;
  }
}

// Returns 0 on success, 1 for non-ASCII, 2 for an operator word.
inline int parse_query(const uint8_t *q, uint64_t n, std::vector<QueryTerm> *terms) {
  for (uint64_t i = 0; i < n; i++)
    if (q[i] >= 0x80) return 1;
  auto ws = [](uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; };
  std::vector<std::string> toks;
  uint64_t i = 0;
  while (i < n) {
    while (i < n && ws(q[i])) i++;
    uint64_t j = i;
    while (j < n && !ws(q[j])) j++;
    const uint64_t w = j - i;
    if ((w == 3 && (!memcmp(q + i, "AND", 3) || !memcmp(q + i, "NOT", 3))) || (w == 2 && !memcmp(q + i, "OR", 2)))
      return 2;
    if (w) analyze_ascii(q + i, w, &toks);
    i = j;
  }
  std::unordered_map<std::string, size_t> pos;
  for (auto &t : toks) {
    auto it = pos.find(t);
    if (it == pos.end()) {
      pos.emplace(t, terms->size());
      terms->push_back(QueryTerm{t, 1.0f});
    } else {
      (*terms)[it->second].boost += 1.0f;
    }
  }
  return 0;
}

inline void term_key(const std::string &t, uint64_t *lo, uint64_t *hi) {
  KeyBuilder kb;
  for (unsigned char c : t) kb.push(c);
  kb.finish(lo, hi);
}

}  // namespace tfidf
