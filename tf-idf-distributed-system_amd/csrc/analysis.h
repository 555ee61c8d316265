// analysis.h — host-side query analysis for tfidf_search (Worker.java:225-227:
// QueryParser("contents", new StandardAnalyzer()).parse(QueryParser.escape(q))).
//
// QueryParser.escape backslash-escapes every query-syntax character
// (\ + - ! ( ) : ^ [ ] " { } ~ * ? | & /), so the parse of an escaped string is
// a flat OR of per-chunk analysed tokens — except for the operator WORDS
// AND / OR / NOT, which escape() leaves alone.  Those are rejected
// (TFIDF_E_UNSUPPORTED_QUERY) rather than silently mis-scored.  Chunks are
// split on the classic QueryParser's whitespace (space, \t, \n, \r, U+3000);
// BooleanQuery.rewrite de-duplicates SHOULD clauses with boost = count.
#pragma once

#include <stdint.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "tfidf_common.h"
#include "unicode_scan.h"

namespace tfidf {

struct QueryTerm {
  std::string term;   // lower-cased analysed token
  float boost;        // occurrence count
};

// StandardAnalyzer over [s, s + n) (unicode_scan.h: the same scanner the
// device runs): lower-cased token strings.  Returns false on malformed UTF-8.
inline bool analyze(const uint8_t *s, uint64_t n, std::vector<std::string> *out) {
  struct StrSink {
    std::string *t;
    void push(uint8_t c) { t->push_back((char)c); }
  };
  uint64_t pos = 0, ts, te;
  bool bad = false;
  while (uc_next_span(UcDecodeSrc{s, n}, n, &pos, n, &ts, &te, &bad)) {
    std::string t;
    StrSink sink{&t};
    const uint64_t cut = uc_token_bytes(s, n, ts, te, sink);
    if (cut < te) pos = cut;
    out->push_back(std::move(t));
  }
  return !bad;
}

// classic QueryParser whitespace: ' ' '\t' '\n' '\r' and U+3000 (E3 80 80)
inline uint32_t qp_ws_len(const uint8_t *q, uint64_t n, uint64_t i) {
  const uint8_t c = q[i];
  if (c == ' ' || c == '\t' || c == '\n' || c == '\r') return 1;
  if (c == 0xE3 && i + 2 < n && q[i + 1] == 0x80 && q[i + 2] == 0x80) return 3;
  return 0;
}

// Returns 0 on success, 1 for malformed UTF-8, 2 for an operator word.
inline int parse_query(const uint8_t *q, uint64_t n, std::vector<QueryTerm> *terms) {
  std::vector<std::string> toks;
  uint64_t i = 0;
  while (i < n) {
    uint32_t w;
    while (i < n && (w = qp_ws_len(q, n, i))) i += w;
    uint64_t j = i;
    while (j < n && !qp_ws_len(q, n, j)) j++;
    const uint64_t len = j - i;
    if ((len == 3 && (!memcmp(q + i, "AND", 3) || !memcmp(q + i, "NOT", 3))) || (len == 2 && !memcmp(q + i, "OR", 2)))
      return 2;
    if (len && !analyze(q + i, len, &toks)) return 1;
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
