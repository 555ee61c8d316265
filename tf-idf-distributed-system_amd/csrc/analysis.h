// analysis.h — host-side query analysis for tfidf_search (Worker.java:225-227:
// QueryParser("contents", new StandardAnalyzer()).parse(QueryParser.escape(q))).
//
// QueryParser.escape backslash-escapes every query-syntax character
// (\ + - ! ( ) : ^ [ ] " { } ~ * ? | & /), so after escaping the only syntax
// left is whitespace and the operator WORDS AND / OR / NOT, which escape()
// leaves alone.  The classic grammar (Lucene 9.8.0 queryparser/classic
// QueryParser.jj, splitOnWhitespace = true, default operator OR) then reads
//
//   Query     := Modifiers Clause ( Conjunction Modifiers Clause )*
//   Conjunction := [ AND | OR ]      Modifiers := [ NOT ]
//   Clause    := TERM                 (a whitespace chunk, escapes removed)
//
// and QueryParserBase.addClause assigns occurs: AND makes the previous clause
// MUST (unless it is MUST_NOT) and the new one MUST; NOT makes the new one
// MUST_NOT; otherwise SHOULD.  A clause is QueryBuilder.createFieldQuery of
// the chunk: no token -> nothing (but AND still marks the previous clause), one
// token -> TermQuery, several -> BooleanQuery of SHOULD TermQuerys
// (analyzeMultiBoolean).  Anything else (leading AND/OR, a trailing operator,
// "NOT NOT", an empty query) is a ParseException -> Worker returns [].
//
// The parsed query is then brought to BooleanQuery.rewrite's fixpoint
// (Lucene 9.8.0 search/BooleanQuery.java rewrite): nested pure disjunctions in
// SHOULD position are flattened; SHOULD clauses and MUST clauses are each
// de-duplicated by summing their boosts (a nested BooleanQuery with one
// distinct token is BoostQuery(term, count)).  The result is a QueryPlan:
// MUST groups (one per distinct MUST clause: its tokens), SHOULD terms,
// MUST_NOT terms; kernels_query.hip scores it.
#pragma once

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "tfidf_common.h"
#include "unicode_scan.h"

namespace tfidf {

constexpr size_t kMaxClauseCount = 1024;   // IndexSearcher.getMaxClauseCount() default

struct PlanTerm {
  std::string term;   // lower-cased analysed token
  float boost;        // product of the clause boost and the token's count in its clause
  uint32_t role;      // kRoleShould / kRoleMust / kRoleNot
  uint32_t group;     // MUST clause index (kRoleMust only)
};

// Terms in kernel order: MUST groups (group 0's terms, group 1's, ...), then
// SHOULD terms (first appearance), then MUST_NOT terms.
struct QueryPlan {
  std::vector<PlanTerm> terms;
  uint32_t n_groups = 0;
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

enum { kQOk = 0, kQBadUtf8 = 1, kQSyntax = 2 };

namespace qp {

enum Tok { T_TERM, T_AND, T_OR, T_NOT };
enum Occur { SHOULD, MUST, MUST_NOT };

// One parsed clause after its own rewrite: distinct tokens with their counts
// (first appearance order).  One distinct token = TermQuery / BoostQuery.
struct Clause {
  Occur occur;
  std::vector<std::pair<std::string, float>> toks;
  // identity for MUST de-duplication (BooleanQuery equality is a multiset of
  // clauses): the sorted (token, count) list; for one token only the token,
  // its count being the BoostQuery boost that the dedupe unwraps and sums
  std::string identity() const {
    if (toks.size() == 1) return "T" + toks[0].first;
    std::vector<std::pair<std::string, float>> s = toks;
    std::sort(s.begin(), s.end());
    std::string id = "B";
    for (auto &t : s) {
      id += t.first;
      id.push_back('\0');
      id += std::to_string((double)t.second);
      id.push_back('\0');
    }
    return id;
  }
};

}  // namespace qp

// Parse + rewrite.  Returns kQOk, kQBadUtf8 (malformed UTF-8) or kQSyntax
// (ParseException / TooManyClauses: the reference answers []).
inline int parse_query(const uint8_t *q, uint64_t n, QueryPlan *plan) {
  using namespace qp;
  // lexer: whitespace-separated chunks; a chunk equal to AND / OR / NOT is the
  // operator token (JavaCC longest match, ties to the earlier-declared operator)
  std::vector<std::pair<uint64_t, uint64_t>> span;
  std::vector<Tok> kind;
  for (uint64_t i = 0; i < n;) {
    uint32_t w;
    while (i < n && (w = qp_ws_len(q, n, i))) i += w;
    if (i >= n) break;
    uint64_t j = i;
    while (j < n && !qp_ws_len(q, n, j)) j++;
    const uint64_t len = j - i;
    Tok t = T_TERM;
    if (len == 3 && !memcmp(q + i, "AND", 3)) t = T_AND;
    else if (len == 2 && !memcmp(q + i, "OR", 2)) t = T_OR;
    else if (len == 3 && !memcmp(q + i, "NOT", 3)) t = T_NOT;
    span.emplace_back(i, len);
    kind.push_back(t);
    i = j;
  }
  std::vector<Clause> clauses;
  bool bad_utf8 = false, too_many = false;
  // QueryParserBase.addClause with operator == OR_OPERATOR
  auto add_clause = [&](bool conj_and, bool mod_not, size_t ti) {
    if (!clauses.empty() && conj_and && clauses.back().occur != MUST_NOT) clauses.back().occur = MUST;
    std::vector<std::string> toks;
    if (!analyze(q + span[ti].first, span[ti].second, &toks)) { bad_utf8 = true; return; }
    if (toks.empty()) return;                         // the analyzer removed everything: q == null
    if (toks.size() > kMaxClauseCount) { too_many = true; return; }   // analyzeMultiBoolean's builder
    Clause c;
    c.occur = mod_not ? MUST_NOT : (conj_and ? MUST : SHOULD);
    std::unordered_map<std::string, size_t> at;       // the nested query's own SHOULD dedupe
    for (auto &t : toks) {
      auto it = at.find(t);
      if (it == at.end()) {
        at.emplace(t, c.toks.size());
        c.toks.emplace_back(t, 1.0f);
      } else {
        c.toks[it->second].second += 1.0f;
      }
    }
    clauses.push_back(std::move(c));
  };
  size_t p = 0;
  const size_t m = kind.size();
  {
    bool mod_not = false;
    if (p < m && kind[p] == T_NOT) { mod_not = true; p++; }
    if (p >= m || kind[p] != T_TERM) return kQSyntax;
    add_clause(false, mod_not, p++);
  }
  while (p < m) {
    bool conj_and = false;
    if (kind[p] == T_AND || kind[p] == T_OR) { conj_and = kind[p] == T_AND; p++; }
    bool mod_not = false;
    if (p < m && kind[p] == T_NOT) { mod_not = true; p++; }
    if (p >= m || kind[p] != T_TERM) return kQSyntax;
    add_clause(conj_and, mod_not, p++);
  }
  if (bad_utf8) return kQBadUtf8;
  if (too_many || clauses.size() > kMaxClauseCount) return kQSyntax;   // getBooleanQuery's builder

  // --- BooleanQuery.rewrite fixpoint ---
  // MUST: de-duplicate identical clauses, summing the unwrapped boosts
  std::vector<size_t> must;
  std::unordered_map<std::string, size_t> must_at;
  std::vector<double> must_boost;
  for (size_t i = 0; i < clauses.size(); i++) {
    if (clauses[i].occur != MUST) continue;
    const std::string id = clauses[i].identity();
    const double u = clauses[i].toks.size() == 1 ? clauses[i].toks[0].second : 1.0;
    auto it = must_at.find(id);
    if (it == must_at.end()) {
      must_at.emplace(id, must.size());
      must.push_back(i);
      must_boost.push_back(u);
    } else {
      must_boost[it->second] += u;
    }
  }
  // SHOULD: nested pure disjunctions flattened, then de-duplicated by term
  std::vector<std::pair<std::string, double>> should;
  std::unordered_map<std::string, size_t> should_at;
  size_t flat = 0, not_clauses = 0;
  for (const Clause &c : clauses) {
    if (c.occur != SHOULD) continue;
    for (auto &t : c.toks) {
      auto it = should_at.find(t.first);
      if (it == should_at.end()) {
        should_at.emplace(t.first, should.size());
        should.emplace_back(t.first, (double)t.second);
      } else {
        should[it->second].second += (double)t.second;
      }
    }
  }
  // the flattening builder holds every SHOULD clause's tokens next to the other
  // clauses (before the flattened duplicates are merged on the next pass)
  {
    std::unordered_map<std::string, int> seen_should;
    for (const Clause &c : clauses)
      if (c.occur == SHOULD) {
        std::string id = c.identity();
        if (seen_should.emplace(id, 1).second) flat += c.toks.size() == 1 ? 1 : c.toks.size();
      }
    std::unordered_map<std::string, int> seen_not;
    for (const Clause &c : clauses)
      if (c.occur == MUST_NOT && seen_not.emplace(c.identity(), 1).second) not_clauses++;
    bool nested_should = false;
    for (const Clause &c : clauses) nested_should |= c.occur == SHOULD && c.toks.size() > 1;
    if (nested_should && flat + must.size() + not_clauses > kMaxClauseCount) return kQSyntax;
  }
  // MUST_NOT: any token of any excluded clause
  std::vector<std::string> excl;
  std::unordered_map<std::string, int> excl_at;
  for (const Clause &c : clauses)
    if (c.occur == MUST_NOT)
      for (auto &t : c.toks)
        if (excl_at.emplace(t.first, 1).second) excl.push_back(t.first);

  plan->terms.clear();
  plan->n_groups = (uint32_t)must.size();
  for (size_t g = 0; g < must.size(); g++) {
    const Clause &c = clauses[must[g]];
    const float B = (float)must_boost[g];
    if (c.toks.size() == 1) {
      plan->terms.push_back(PlanTerm{c.toks[0].first, B, kRoleMust, (uint32_t)g});
    } else {
      for (auto &t : c.toks) {
        volatile float bt = B * t.second;             // BoostQuery boost x inner BoostQuery boost (float)
        plan->terms.push_back(PlanTerm{t.first, (float)bt, kRoleMust, (uint32_t)g});
      }
    }
  }
  for (auto &s : should) plan->terms.push_back(PlanTerm{s.first, (float)s.second, kRoleShould, 0});
  for (auto &x : excl) plan->terms.push_back(PlanTerm{x, 1.0f, kRoleNot, 0});
  return kQOk;
}

inline void term_key(const std::string &t, uint64_t *lo, uint64_t *hi, uint64_t seed = 0) {
  KeyBuilder kb;
  for (unsigned char c : t) kb.push(c);
  kb.finish(lo, hi, seed);
}

}  // namespace tfidf
