/*
 * tfidf_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C, single-threaded restatement of the reference's hot path, which
 * lives in Apache Lucene 9.8.0 (org.apache.lucene:lucene-core /
 * lucene-queryparser / lucene-analysis-common 9.8.0, pinned at
 * TF-IDF-System-Core/pom.xml:77-93; not vendored under /root/reference).
 * Call sites restated:
 *   Worker.addDocToIndex  TF-IDF-System-Core/src/main/java/me/zookeeper/leader_election/worker/Worker.java:190-220
 *   Worker.searchIndex    .../worker/Worker.java:222-241
 *   Leader.start merge    .../leader/Leader.java:39-92
 *
 * Pinned by: tests/golden/lucene_sample8.json, decoded from the reference's
 * committed Lucene 9.8.0 index (TF, DF, norm bytes, docCount, sumTotalTermFreq,
 * sumDocFreq).  BM25 scores are NOT pinned by any reference artefact
 * ("parity unpinned" for scores).
 *
 * ONLY tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.  The
 * product (libtfidf) never links or calls it.
 */
#ifndef TFIDF_ORACLE_H
#define TFIDF_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_OK 0
#define ORC_E_ARG (-1)
#define ORC_E_UNSUPPORTED (-2) /* malformed UTF-8 */
#define ORC_E_NOMEM (-3)
#define ORC_E_CAP (-4)         /* caller buffer too small; *n_out = needed */
#define ORC_E_SYNTAX (-5)      /* QueryParser ParseException / TooManyClauses (Worker answers []) */

/* StandardTokenizer (UAX#29 JFlex grammar of Lucene 9.8).
 * Writes token start offsets / lengths (into the ORIGINAL bytes; lower-case
 * folding, orc_lower_utf8, is applied by callers).  Returns the number
 * of tokens (may exceed cap: only the first cap are written), or
 * ORC_E_UNSUPPORTED for malformed UTF-8. */
int64_t orc_tokenize(const uint8_t *s, uint64_t n, uint32_t max_token_len,
                     uint32_t *starts, uint32_t *lens, uint64_t cap);
/* The full-Unicode rules (orc_tokenize uses them when a byte >= 0x80 is
 * present; exported so tests can run them on ASCII too).  Spans are in bytes;
 * max_token_len counts UTF-16 units.  ORC_E_UNSUPPORTED = malformed UTF-8. */
int64_t orc_tokenize_unicode(const uint8_t *s, uint64_t n, uint32_t max_token_len,
                             uint32_t *starts, uint32_t *lens, uint64_t cap);
/* LowerCaseFilter on one token's UTF-8 (dst >= 2 * len bytes); returns length. */
uint64_t orc_lower_utf8(const uint8_t *src, uint64_t len, uint8_t *dst);

/* SmallFloat.intToByte4 / byte4ToInt (BM25Similarity.computeNorm, LENGTH_TABLE). */
uint8_t orc_int_to_byte4(int32_t i);
int32_t orc_byte4_to_int(uint8_t b);

typedef struct orc_index orc_index;

orc_index *orc_create(float k1, float b);
void orc_destroy(orc_index *ix);
/* updateDocument(Term("path", key), doc): replaces a live doc with the same key. */
int orc_add_doc(orc_index *ix, const uint8_t *key, uint64_t key_len,
                const uint8_t *text, uint64_t n);
int orc_commit(orc_index *ix);

uint64_t orc_num_docs(const orc_index *ix);      /* live docs (maxDoc after compaction) */
uint64_t orc_doc_count(const orc_index *ix);     /* docs with >= 1 token */
uint64_t orc_sum_ttf(const orc_index *ix);
uint64_t orc_num_terms(const orc_index *ix);
uint32_t orc_doc_len(const orc_index *ix, uint64_t doc);
/* Committed docs whose text is not valid UTF-8 (indexed empty); returns the count. */
uint64_t orc_malformed_docs(const orc_index *ix, uint64_t *docs, uint64_t cap);
uint8_t orc_doc_norm(const orc_index *ix, uint64_t doc);
/* key of doc; returns length, copies up to cap bytes */
uint64_t orc_doc_key(const orc_index *ix, uint64_t doc, uint8_t *buf, uint64_t cap);
/* Distinct terms of a doc sorted by bytes: terms NUL-separated into buf.
 * Returns the number of distinct terms (or ORC_E_CAP with nothing written). */
int64_t orc_doc_terms(const orc_index *ix, uint64_t doc, char *buf, uint64_t buf_cap,
                      uint32_t *tfs, uint64_t cap);
int64_t orc_df(const orc_index *ix, const uint8_t *term, uint64_t len);
/* Vocabulary export: all terms NUL-separated (index order) + df. */
int64_t orc_vocab(const orc_index *ix, char *buf, uint64_t buf_cap, uint32_t *df, uint64_t cap);

/* GLOBAL-stats override (the 1-worker semantics of a sharded corpus):
 * per-term df by string, plus docCount / sumTotalTermFreq.  Pass
 * doc_count == 0 to revert to the shard's own statistics. */
int orc_set_global_stats(orc_index *ix, uint64_t doc_count, uint64_t sum_ttf);
int orc_set_global_df(orc_index *ix, const uint8_t *term, uint64_t len, uint64_t df);

/* Worker.searchIndex: parse(escape(q)) (operator words AND / OR / NOT kept)
 * -> rewritten BooleanQuery -> BM25 scores -> hits ordered (score desc, doc
 * asc).  k == 0 returns all hits (searcher.search(q, MAX)).  Returns ORC_OK /
 * ORC_E_UNSUPPORTED / ORC_E_SYNTAX / ORC_E_CAP (n_out = needed). */
int orc_search(const orc_index *ix, const uint8_t *q, uint64_t q_len, uint32_t k,
               uint32_t *docs, float *scores, uint64_t cap, uint64_t *n_out);

/* SHOULD terms of the parsed + rewritten query (nested disjunctions
 * flattened, duplicates merged, first appearance order) NUL-separated + boost
 * (occurrence count).  Returns #terms or error. */
int64_t orc_query_terms(const uint8_t *q, uint64_t q_len, char *buf, uint64_t buf_cap,
                        float *boosts, uint64_t cap);

/* BM25 pieces in Java float/double order (BM25Similarity 9.8.0). */
float orc_idf(uint64_t doc_freq, uint64_t doc_count);
float orc_avgdl(uint64_t sum_ttf, uint64_t doc_count);
void orc_norm_cache(float k1, float b, float avgdl, float cache[256]);
float orc_bm25(float weight, uint32_t tf, float norm_inverse);

/* Leader.start merge: names (concatenated, offsets[n+1]) with double scores in
 * worker-response order -> distinct names sorted by String.compareTo (UTF-16
 * code units) with Double::sum totals.  Output: index of first occurrence of
 * each distinct name in sorted order + sums.  Returns #distinct. */
int64_t orc_leader_merge(const uint8_t *names, const uint64_t *offsets, uint64_t n,
                         const double *scores, uint64_t *out_first, double *out_sum);

/* CPU baseline only (bench.py cpu_baseline; never the checker): n_threads
 * POSIX threads, thread t indexes documents [t*n/T, (t+1)*n/T) of the corpus
 * (text + offsets[n_docs + 1]) into ITS OWN index — the reference's N-worker
 * layout, one IndexWriter per worker (Worker.java:67-88) — keyed by the
 * decimal document number, and commits it.  *seconds = wall time of the
 * parallel region (thread start to the last commit); *sum_ttf = tokens
 * indexed over all threads (a check that the work was done).  Returns ORC_OK. */
int orc_bulk_build(const uint8_t *text, const uint64_t *offsets, uint64_t n_docs, uint32_t n_threads,
                   double *seconds, uint64_t *sum_ttf);

#ifdef __cplusplus
}
#endif
#endif
