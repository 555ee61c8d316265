/*
 * tfidf.h — C ABI of libtfidf, the MI355X-native TF-IDF/BM25 engine.
 *
 * Drop-in boundary for the reference's hot path (kheder-hassoun/
 * Tf-IDF-Distributed-System, Java + Lucene 9.8.0).  The reference has no
 * plugin API: the path sits behind direct Lucene calls in two Java methods
 * and one merge loop.  Each entry point below names the reference interface
 * it replaces (paths relative to TF-IDF-System-Core/src/main/java/):
 *
 *   tfidf_create / tfidf_destroy
 *       me/zookeeper/leader_election/worker/Worker.java:67-73
 *       (FSDirectory.open + new IndexWriter(dir, IndexWriterConfig(new StandardAnalyzer())))
 *   tfidf_add_docs / tfidf_add_docs_device
 *       Worker.java:190-220 addDocToIndex -> indexWriter.updateDocument(Term("path", rel), doc)
 *       (called from the Files.walk loop Worker.java:77-86 and upload Worker.java:136-139)
 *   tfidf_commit
 *       Worker.java:88 and :138 indexWriter.commit() (+ DirectoryReader.open at :223 sees it)
 *   tfidf_search / tfidf_search_batch
 *       Worker.java:222-241 searchIndex: QueryParser("contents", StandardAnalyzer)
 *       .parse(QueryParser.escape(q)); searcher.search(query, Integer.MAX_VALUE)
 *   tfidf_doc_key
 *       Worker.java:235-236 searcher.doc(sd.doc).get("path")
 *   tfidf_stats
 *       Worker.java:147-172 /worker/index-size (device bytes) + Lucene CollectionStatistics
 *   tfidf_vocab_* / tfidf_set_global_*
 *       no reference counterpart: GLOBAL statistics across GPU shards (the
 *       reference's 1-worker semantics, Leader.java:39-92 with one worker)
 *   tfidf_leader_merge
 *       me/zookeeper/leader_election/leader/Leader.java:73-88 (sum per name, TreeMap order)
 *   tfidf_node_* / tfidf_dist_* / tfidf_comm_*
 *       Leader.java:39-92 start (fan-out :51-70 over Worker.java:222-241, merge :73-88)
 *       with the workers as GPU shards and RCCL collectives in place of HTTP
 *
 * Conventions: every call returns an int status (TFIDF_OK == 0); the message
 * of the last failure on the calling thread is tfidf_last_error().  Buffers
 * are caller-owned and only borrowed for the duration of a call.
 * Threading (Worker.java:223 opens a DirectoryReader on the last commit per
 * request while uploads commit beside it, :136-139): every commit publishes an
 * immutable, refcounted snapshot.  Searches and the other read calls run on
 * the snapshot published when they start, concurrently with each other (each
 * on its own stream and scratch) and with tfidf_add_docs / tfidf_commit on
 * another thread, and never wait for a commit; a snapshot is freed, or rebuilt
 * by a later commit, when its last reader leaves.  Documents added after a
 * commit are invisible to searches until the next commit.  Writers (add_docs,
 * commit, clear, load, the GLOBAL statistics setters) serialise among
 * themselves (Worker.java:136 synchronized(indexWriter)).
 * Scores are IEEE float32 bit-identical to Lucene 9.8.0 BM25Similarity
 * (k1 = 1.2, b = 0.75); hits are ordered by (score desc, doc asc).
 */
#ifndef TFIDF_H
#define TFIDF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TFIDF_OK 0
#define TFIDF_E_INVALID_ARG 1
#define TFIDF_E_HIP 2
#define TFIDF_E_OOM 3
#define TFIDF_E_UNSUPPORTED_INPUT 4 /* tf >= 2^24 (a malformed UTF-8 document is indexed empty, see
                                       tfidf_malformed_docs) */
#define TFIDF_E_UNSUPPORTED_QUERY 5 /* malformed UTF-8 query */
#define TFIDF_E_CAPACITY 6          /* vocabulary capacity exceeded */
#define TFIDF_E_STATE 7             /* e.g. search before commit */
#define TFIDF_E_BUFFER 8            /* caller buffer too small; *n_out holds the size needed */
#define TFIDF_E_NO_DEVICE 9
#define TFIDF_E_QUERY_SYNTAX 10     /* QueryParser ParseException / TooManyClauses (Worker.java:182-185 -> []):
                                       empty query, leading AND/OR, trailing or doubled operator word */

#define TFIDF_STATS_SHARD 0  /* per-shard statistics: the reference's N-worker semantics */
#define TFIDF_STATS_GLOBAL 1 /* statistics imported from all shards: 1-worker semantics */

/* Inverted-index layout built by tfidf_commit (results are identical). */
#define TFIDF_INVERSION_AUTO 0  /* block-major unless its (docs/8192 + 1) x 2^vocab_capacity_log2 count table
                                   outgrows the CSR, or vocab_capacity_log2 > 21 (huge vocabularies), or the
                                   corpus is a few very long documents (fewer (block, range) tiles than CUs,
                                   >= 64 KB per document: books) */
#define TFIDF_INVERSION_BLOCK 1 /* block-major: postings grouped by 8192-doc block, then term */
#define TFIDF_INVERSION_TERM 2  /* term-major: postings grouped by term, docs ascending (sort-based) */

typedef struct tfidf_index tfidf_index;

typedef struct tfidf_config {
  float k1;                     /* BM25 k1, default 1.2f (BM25Similarity()) */
  float b;                      /* BM25 b,  default 0.75f */
  int32_t stats_mode;           /* TFIDF_STATS_SHARD (default) or TFIDF_STATS_GLOBAL */
  int32_t device;               /* HIP device ordinal */
  uint32_t vocab_capacity_log2; /* dictionary slots = 2^x, x in [10, 26]; default 18 (<= ~200k terms);
                                   x > 21 implies the term-major inversion */
  uint32_t max_token_len;       /* StandardAnalyzer.DEFAULT_MAX_TOKEN_LENGTH = 255 (only value supported) */
  int32_t inversion;            /* TFIDF_INVERSION_AUTO (default), _BLOCK or _TERM */
} tfidf_config;

typedef struct tfidf_index_stats {
  uint64_t num_docs;      /* live documents (maxDoc after compaction) */
  uint64_t doc_count;     /* documents with >= 1 token (CollectionStatistics.docCount) */
  uint64_t sum_ttf;       /* sumTotalTermFreq */
  uint64_t num_terms;     /* distinct terms in this shard */
  uint64_t nnz;           /* (doc, term) postings = sumDocFreq */
  uint64_t device_bytes;  /* HBM held by the index (feeds /worker/index-size) */
  uint64_t long_docs;     /* documents indexed by the long-document path */
  uint64_t text_bytes;    /* corpus bytes resident on the device */
  uint64_t term_major;    /* 1 if the last commit built the term-major layout (TFIDF_INVERSION_TERM) */
  uint64_t pack_docs;     /* documents per tokenizer window in the last commit (1 = one per window) */
  uint64_t pack_retried;  /* documents the packed windows handed to the one-per-window pass */
  uint64_t unicode_docs;  /* documents (window <= 4 KB) the ASCII wave path found non-ASCII text in */
  uint64_t long_chunked;  /* long documents indexed chunk-parallel (the rest of long_docs: k_tokenize_long) */
  uint64_t malformed_docs;/* documents that are not valid UTF-8, indexed empty (tfidf_malformed_docs) */
  uint64_t hash_seed;     /* seed of the hashed term keys (> 16-byte terms, > 14-byte non-ASCII ones); 0 unless a
                             hash collision was detected and the build redone (term identity stays
                             exact: every merge under a hashed key compares the strings) */
  uint64_t hash_rebuilds; /* seed attempt in force (0 = first seed): builds redone in the last commit because of
                             a hash collision, plus the floor set by tfidf_set_hash_attempt */
  uint64_t coalesced_batches;  /* tfidf_search_coalesced: batches run / queries served (index lifetime) */
  uint64_t coalesced_queries;
  uint64_t unit_batches;   /* batched top-k searches scored by query units (k_score_units) / units run */
  uint64_t unit_count;
  uint64_t fused_queries;  /* tfidf_search top-k calls served by the one-launch fused path (index lifetime) */
  uint64_t unicode_wave_docs;  /* of unicode_docs: those the wave rules took (non-ASCII letters that are
                                  ALetter and lower case only); the rest went to the Unicode wave path */
} tfidf_index_stats;

/* Per-phase device times of the last commit, measured with HIP events on the
 * index's stream around each kernel. */
typedef struct tfidf_commit_timing {
  float ms_total;
  float ms_tokenize;   /* tfidf_tokenize_count: text -> per-doc TF rows (CSR) */
  float ms_long;       /* long-document path */
  float ms_df;         /* per (doc block, term range) DF histograms */
  float ms_blockscan;  /* DF = sum over doc blocks + per-block posting offsets (scan over slots) */
  float ms_colscan;    /* exclusive scan of block totals -> block bases */
  float ms_scatter;    /* CSR -> block-segmented inverted postings */
  uint64_t text_bytes;
  uint64_t num_docs;
  uint64_t nnz;
} tfidf_commit_timing;

const char *tfidf_version(void);
const char *tfidf_last_error(void);
int tfidf_config_init(tfidf_config *cfg);

int tfidf_create(const tfidf_config *cfg, tfidf_index **out);
int tfidf_destroy(tfidf_index *ix);

/* Host corpus: n_docs documents, document i = utf8[offsets[i] .. offsets[i+1]).
 * keys (may be NULL) = relative paths, key i = keys[key_offsets[i] .. key_offsets[i+1]);
 * a key already present replaces that document (updateDocument by Term("path", key)).
 * With keys == NULL the key of a document is its decimal ordinal in this index.
 * Bytes reach HBM through two pinned staging buffers (host copy of one overlapped
 * with the DMA of the other); the call returns once they are resident. */
int tfidf_add_docs(tfidf_index *ix, const uint8_t *utf8, const uint64_t *offsets, uint64_t n_docs,
                   const uint8_t *keys, const uint64_t *key_offsets);
/* Drop every staged and committed document (the index is empty, as after
 * tfidf_create); device and pinned staging buffers are kept for reuse. */
int tfidf_clear(tfidf_index *ix);
/* Device-resident corpus (e.g. produced by tfidf_synth_corpus): copied device-to-device. */
int tfidf_add_docs_device(tfidf_index *ix, const void *d_utf8, const void *d_offsets, uint64_t n_docs,
                          uint64_t total_bytes);

int tfidf_commit(tfidf_index *ix);
/* GLOBAL statistics match terms across shards by their keys, so every shard
 * must hash its long / non-ASCII terms with one seed.  A commit tries seed
 * attempts 0, 1, 2, 3 in turn (the next one after a detected collision);
 * this sets the attempt the following commits start from (0..3; 0 = the
 * default).  Multi-GPU: the ranks agree on the highest attempt any shard
 * needed and re-commit under it (tfidf_amd/distributed.py global_commit).
 * No reference counterpart: each Lucene worker is independent (Leader.java:67-69). */
int tfidf_set_hash_attempt(tfidf_index *ix, uint32_t attempt);

/* Persistence (the reference's FSDirectory index, Worker.java:67-73).  tfidf_save
 * writes the staged corpus (text, offsets, document keys, replace-by-key
 * liveness) to `path` (atomically: path.tmp, then rename).  tfidf_load stages a
 * saved file into an EMPTY index (same vocab_capacity_log2); call tfidf_commit
 * afterwards (more documents may be added first, replacing by key as usual).
 * The inverted index itself is rebuilt by the commit rather than stored. */
int tfidf_save(tfidf_index *ix, const char *path);
int tfidf_load(tfidf_index *ix, const char *path);
int tfidf_get_commit_timing(const tfidf_index *ix, tfidf_commit_timing *out);
int tfidf_stats(const tfidf_index *ix, tfidf_index_stats *out);

/* Single query. k == 0 returns all hits (searcher.search(q, Integer.MAX_VALUE)).
 * doc_ids are local document ordinals; scores are float32. */
int tfidf_search(tfidf_index *ix, const uint8_t *q, uint64_t q_len, uint32_t k, uint32_t *doc_ids,
                 float *scores, uint64_t cap, uint64_t *n_out);
/* n_q queries; query i = q_utf8[q_offsets[i] .. q_offsets[i+1]).  1 <= k <= 1024.
 * Outputs are n_q x k (row i holds counts[i] valid hits). */
/* Concurrent single top-k searches (Worker.processDocuments on concurrent
 * request threads, Worker.java:175-186): same arguments and results as
 * tfidf_search with 1 <= k <= 1024, but callers arriving together are served
 * by ONE batched scoring launch (the first waits wait_us for companions).
 * Thread-safe; a caller blocks until its own results are written. */
int tfidf_search_coalesced(tfidf_index *ix, const uint8_t *q, uint64_t q_len, uint32_t k, uint32_t *doc_ids,
                           float *scores, uint64_t cap, uint64_t *n_out, uint32_t wait_us);
int tfidf_search_batch(tfidf_index *ix, const uint8_t *q_utf8, const uint64_t *q_offsets, uint32_t n_q,
                       uint32_t k, uint32_t *doc_ids, float *scores, uint32_t *counts);
/* Readers (Worker.java:223 DirectoryReader.open per request; the hits' stored
 * "path" fields are read from the same reader, :234-238): a reader pins the
 * snapshot published when it is opened, so doc ids it returns map to keys
 * with tfidf_reader_doc_key even while later commits publish other snapshots.
 * tfidf_reader_search: as tfidf_search, on the reader's snapshot.
 * tfidf_reader_info: the snapshot's commit generation (1, 2, ... per
 * successful commit) and document count.  A reader may be used from several
 * threads; close it once (its snapshot is released with the last user). */
typedef struct tfidf_reader tfidf_reader;
int tfidf_reader_open(tfidf_index *ix, tfidf_reader **out);
int tfidf_reader_close(tfidf_reader *rd);
int tfidf_reader_info(const tfidf_reader *rd, uint64_t *generation, uint64_t *num_docs);
int tfidf_reader_search(tfidf_reader *rd, const uint8_t *q, uint64_t q_len, uint32_t k, uint32_t *doc_ids,
                        float *scores, uint64_t cap, uint64_t *n_out);
int tfidf_reader_doc_key(const tfidf_reader *rd, uint64_t doc, uint8_t *buf, uint64_t cap, uint64_t *n_out);
/* tfidf_doc_keys of the reader's snapshot (offsets[num_docs + 1] of tfidf_reader_info). */
int tfidf_reader_doc_keys(const tfidf_reader *rd, uint8_t *buf, uint64_t cap, uint64_t *offsets, uint64_t *n_bytes);
/* Per-query device time of the last search call on this index (HIP events on the search's stream). */
int tfidf_last_search_ms(const tfidf_index *ix, float *ms_scoring, float *ms_total);
/* Device-time measurement of searches (HIP events around scoring; on by
 * default).  Off for serving: the three event records cost ~17 us per single
 * query (cfg 2: 72 -> 55 us p50); tfidf_last_search_ms then reports -1. */
int tfidf_set_query_timing(tfidf_index *ix, int on);

/* ---- device-resident results (multi-GPU orchestration; no reference
 * counterpart: they feed the RCCL all-gather that replaces Leader.java:51-70) ----
 * Merge keys: (float32 score bits << 32) | ~(doc_base + doc) as u64 — BM25
 * scores are > 0, so descending key order is (score desc, doc asc); 0 = empty.
 * tfidf_search_batch_keys_device: n_q x k keys into caller device memory
 *   (a query that does not parse has none).
 * tfidf_search_all_keys_device: every hit of one query, ordered, into caller
 *   device memory of cap >= num_docs keys; *n_out = hits.
 * Both return after the keys are written (the index's stream is synchronised). */
int tfidf_search_batch_keys_device(tfidf_index *ix, const uint8_t *q_utf8, const uint64_t *q_offsets, uint32_t n_q,
                                   uint32_t k, uint64_t doc_base, void *d_keys);
int tfidf_search_all_keys_device(tfidf_index *ix, const uint8_t *q, uint64_t q_len, uint64_t doc_base, void *d_keys,
                                 uint64_t cap, uint64_t *n_out);
/* Issue the index's device work on the caller's stream (a hipStream_t, e.g.
 * torch.cuda.current_stream().cuda_stream; NULL = the legacy default stream),
 * or back on the index's own stream with TFIDF_OWN_STREAM.  Pending work on
 * the previous stream is finished first. */
#define TFIDF_OWN_STREAM ((void *)-1)
int tfidf_set_stream(tfidf_index *ix, void *stream);

int tfidf_doc_key(const tfidf_index *ix, uint64_t doc, uint8_t *buf, uint64_t cap, uint64_t *n_out);
/* Every committed document's key (Worker.java:214 StringField "path"), in doc
 * order: bytes concatenated into buf, offsets[num_docs + 1]; TFIDF_E_BUFFER with
 * *n_bytes = size needed when cap is too small.  num_docs is that of the
 * snapshot published at the call: beside concurrent commits, size offsets from
 * a reader (tfidf_reader_doc_keys). */
int tfidf_doc_keys(const tfidf_index *ix, uint8_t *buf, uint64_t cap, uint64_t *offsets, uint64_t *n_bytes);
int tfidf_doc_len(tfidf_index *ix, uint64_t doc, uint32_t *len, uint8_t *norm);
/* Documents of the last commit whose bytes are not valid UTF-8 (where the
 * reference's Files.readString throws MalformedInputException and Tika
 * extracts the text instead, Worker.java:199-211): they are indexed as empty
 * documents (no tokens, norm 0) rather than failing the commit.  Committed doc
 * ids, ascending; *n_out = count (TFIDF_E_BUFFER if cap is too small).  A
 * caller with a text extractor re-adds the extracted text under the same key
 * (replace-by-key) and commits again. */
int tfidf_malformed_docs(const tfidf_index *ix, uint64_t *docs, uint64_t cap, uint64_t *n_out);
/* Distinct terms of one document: NUL-separated strings (sorted by bytes) + tf. */
int tfidf_doc_terms(tfidf_index *ix, uint64_t doc, char *terms, uint64_t terms_cap, uint32_t *tfs,
                    uint64_t cap, uint64_t *n_out);
int tfidf_term_df(tfidf_index *ix, const uint8_t *term, uint64_t len, uint64_t *df_local,
                  uint64_t *df_effective);

/* ---- GLOBAL statistics across shards (no reference counterpart) ----
 * Term-ownership exchange (used by the multi-GPU orchestration; O(vocabulary)
 * per rank, no sort).  With a caller's stream (tfidf_set_stream: the
 * collective stream) the three device calls are ASYNCHRONOUS on it: the
 * caller's device buffers must stay allocated until that stream reaches the
 * work (true when they come from an allocator that orders them on that
 * stream, as torch's caching allocator does), and the exchange needs one host
 * read — the split sizes.  On the index's own stream each call returns after
 * its device work is done, so the buffers may be freed as soon as it returns.
 * 1. tfidf_vocab_partition_device: this shard's vocabulary as records
 *    (lo, hi, df: 3 x u64 each) grouped by owner rank (a hash of the term key
 *    mod n_ranks) into d_records; d_counts (device, n_ranks x u64) = records
 *    per owner; *n_out = records (the shard's vocabulary size, host-known).
 * 2. caller all-to-alls the records to their owners (RCCL), then the owner
 *    calls tfidf_vocab_reduce_device on everything it received: d_df_out
 *    (u32 per record, same order) = df summed over identical terms;
 *    d_n_unique (device u64, may be NULL) = distinct terms this rank owns.
 * 3. caller all-to-alls the answers back (reverse split sizes), sums
 *    {doc_count, sum_ttf} over ranks, and tfidf_set_global_df_device imports
 *    the answers (in the record order step 1 produced); its host mirror is
 *    copied in the background and waited for by the next search.
 * Canonical-vocabulary form (sorted union; kept for tools and tests):
 * 1. tfidf_vocab_export_device: this shard's term keys (16 B each, sorted
 *    ascending as (hi, lo)) and local df into caller device buffers.
 * 2. caller all-gathers the key lists (RCCL), then
 *    tfidf_vocab_canonicalize_device: sorted union of all shards' keys ->
 *    canonical term ids; fills d_df_canonical (u32[n_canonical]) with this
 *    shard's df in canonical order (zero elsewhere).
 * 3. caller all-reduces d_df_canonical and {doc_count, sum_ttf} (RCCL SUM), then
 *    tfidf_set_global_stats_device imports them. */
int tfidf_vocab_partition_device(tfidf_index *ix, uint32_t n_ranks, void *d_records, uint64_t cap, void *d_counts,
                                 uint64_t *n_out);
int tfidf_vocab_reduce_device(tfidf_index *ix, const void *d_records, uint64_t n, void *d_df_out, void *d_n_unique);
int tfidf_set_global_df_device(tfidf_index *ix, const void *d_df, uint64_t n, uint64_t doc_count,
                               uint64_t sum_ttf);
int tfidf_vocab_size(const tfidf_index *ix, uint64_t *n);
/* Host copy of this shard's vocabulary with the statistics in force: term
 * keys (lo, hi: 2 x u64 each, sorted ascending as (hi, lo)), the shard's own
 * docFreq and the effective one (the GLOBAL df after an exchange, else the
 * shard's own).  Any output may be NULL; *n_out = the vocabulary size
 * (TFIDF_E_BUFFER if it exceeds cap). */
int tfidf_vocab_export(tfidf_index *ix, uint64_t *keys, uint32_t *df_local, uint32_t *df_effective, uint64_t cap,
                       uint64_t *n_out);
int tfidf_vocab_export_device(tfidf_index *ix, void *d_keys, void *d_df, uint64_t cap, uint64_t *n_out);
int tfidf_vocab_canonicalize_device(tfidf_index *ix, const void *d_all_keys, uint64_t n_all,
                                    void *d_df_canonical, uint64_t cap, uint64_t *n_canonical);
int tfidf_set_global_stats_device(tfidf_index *ix, const void *d_df_canonical, uint64_t n_canonical,
                                  uint64_t doc_count, uint64_t sum_ttf);
/* Host-buffer form of the same import: df for arbitrary keys (2 x u64 per key: lo, hi). */
int tfidf_set_global_stats(tfidf_index *ix, const uint64_t *keys_lohi, const uint64_t *df, uint64_t n,
                           uint64_t doc_count, uint64_t sum_ttf);
int tfidf_clear_global_stats(tfidf_index *ix);

/* Term key of an analysed (lower-cased) token, as the device computes it. */
int tfidf_term_key(const uint8_t *term, uint64_t len, uint64_t *lo, uint64_t *hi);

/* StandardAnalyzer (Worker.java:71,225: StandardTokenizer + LowerCaseFilter,
 * full Unicode, maxTokenLength 255) on the host, the same scanner the index
 * build runs on the device: NUL-terminated lower-cased UTF-8 tokens in order.
 * TFIDF_E_BUFFER with *n_bytes = size needed when cap is too small;
 * TFIDF_E_UNSUPPORTED_INPUT for malformed UTF-8. */
int tfidf_analyze(const uint8_t *text, uint64_t len, char *out, uint64_t cap, uint64_t *n_tokens,
                  uint64_t *n_bytes);

/* Leader.start merge (Leader.java:73-88): names (concatenated, offsets[n+1])
 * with double scores in worker-response order -> distinct names sorted by
 * String.compareTo (UTF-16 code units) with Double::sum totals.  out_first[i]
 * = index of the first occurrence of the i-th distinct name.  n_out = #distinct. */
int tfidf_leader_merge(const uint8_t *names, const uint64_t *offsets, uint64_t n, const double *scores,
                       uint64_t *out_first, double *out_sum, uint64_t *n_out);
/* Stable permutation of n UTF-8 names in String.compareTo (UTF-16) order (the
 * TreeMap order of Leader.java:80-88; the multi-GPU name table). */
int tfidf_sort_names(const uint8_t *names, const uint64_t *offsets, uint64_t n, uint64_t *perm);

/* ==========================================================================
 * Node level: documents sharded over GPUs, one shard (tfidf_index) per GPU.
 *
 * Replaces the reference's fan-out + merge, Leader.java:39-92 (POST
 * {worker}/worker/process to every registered worker, :51-70; merge by name,
 * :73-88) over each worker's Worker.java:222-241 searchIndex, with
 * collectives between the shards (RCCL over xGMI on one MI355X node):
 *   GLOBAL statistics (cfg.stats_mode TFIDF_STATS_GLOBAL: the reference's
 *     1-worker results on a sharded corpus): per commit, each term's (key, df)
 *     records go to an owner rank (all-to-all), the owner sums df and answers
 *     (all-to-all back); docCount / sumTotalTermFreq summed; per query, every
 *     shard's top-k as merge keys, all-gathered and merged on the device.
 *     Global doc id = shard base + local id (contiguous shards): (score desc,
 *     doc asc) is the single-index order.  At most 2^32 documents per node.
 *   SHARD statistics (TFIDF_STATS_SHARD: the reference's N-worker results):
 *     every shard scores with its own statistics and returns ALL its hits;
 *     the hits are summed per document name in double in rank (= worker
 *     response) order (HashMap.merge Double::sum, Leader.java:73-77) and
 *     ordered by String.compareTo (TreeMap, :80-88).
 *
 * Two process models, one orchestration (the code below the ABI is the same):
 *   (1) tfidf_node: ONE process owns every GPU of a device list (SURVEY §8b:
 *       "one JVM owns all 8 GPUs"); one host thread per shard; collectives
 *       over an RCCL communicator of the devices (ncclCommInitAll), or an
 *       in-process host transport when a device repeats (tests) or
 *       TFIDF_NODE_INPROC is asked for.
 *   (2) SPMD, one process per GPU: each rank creates its own tfidf_index and a
 *       tfidf_comm (built-in RCCL from a unique id the caller broadcasts, or
 *       the caller's own collectives through tfidf_collectives), and calls the
 *       tfidf_dist_* functions collectively (every rank, same order).
 * ========================================================================== */
typedef struct tfidf_comm tfidf_comm;
typedef struct tfidf_node tfidf_node;

#define TFIDF_COLL_HOST 0    /* collective buffers are host memory (gloo / MPI / sockets ...) */
#define TFIDF_COLL_DEVICE 1  /* device memory of the rank's GPU, ordered on `stream` (a hipStream_t) */

/* Caller-supplied collectives (the transport of process model (2) when the
 * built-in RCCL communicator is not used).  Each returns 0 on success.
 *   all_gather   : recv[r * bytes .. (r + 1) * bytes) = rank r's send, bytes each
 *   all_to_all_v : send_bytes[r] bytes at send + send_offs[r] go to rank r;
 *                  recv_bytes[r] bytes from rank r land at recv + recv_offs[r]
 * Buffers may be NULL when their byte counts are 0.  With TFIDF_COLL_DEVICE the
 * call may be asynchronous on `stream`; with TFIDF_COLL_HOST it must be complete
 * on return. */
typedef struct tfidf_collectives {
  void *ctx;
  int32_t memory;              /* TFIDF_COLL_HOST or TFIDF_COLL_DEVICE */
  int (*all_gather)(void *ctx, const void *send, void *recv, uint64_t bytes, void *stream);
  int (*all_to_all_v)(void *ctx, const void *send, const uint64_t *send_bytes, const uint64_t *send_offs,
                      void *recv, const uint64_t *recv_bytes, const uint64_t *recv_offs, void *stream);
} tfidf_collectives;

/* A communicator over the caller's collectives (the table is copied). */
int tfidf_comm_create(int32_t rank, int32_t world, const tfidf_collectives *coll, tfidf_comm **out);
/* Built-in RCCL communicator (librccl of the HIP runtime the library runs on,
 * loaded at first use): rank 0 calls tfidf_rccl_unique_id, the caller sends the
 * 128 bytes to every rank (its own channel), then every rank calls
 * tfidf_comm_init_rccl with its rank and GPU (collective). */
int tfidf_rccl_unique_id(uint8_t id[128]);
int tfidf_comm_init_rccl(const uint8_t id[128], int32_t rank, int32_t world, int32_t device, tfidf_comm **out);
/* `world` communicators of one process sharing an in-process host transport
 * (comms[0 .. world-1], rank i = comms[i]); each rank's calls run on its own
 * thread.  The transport tfidf_node uses when shards share a device. */
int tfidf_comm_create_inproc(int32_t world, tfidf_comm **comms);
int tfidf_comm_destroy(tfidf_comm *c);
int tfidf_comm_info(const tfidf_comm *c, int32_t *rank, int32_t *world, int32_t *transport);
#define TFIDF_TRANSPORT_CALLBACK 0
#define TFIDF_TRANSPORT_RCCL 1
#define TFIDF_TRANSPORT_INPROC 2
/* Transport check (no index needed): an all-gather of each rank's id and an
 * all-to-all-v of rank-tagged bytes through the communicator, verified on
 * every rank.  Collective. */
int tfidf_comm_selftest(tfidf_comm *c);

/* ---- process model (2): per-rank calls, collective over the communicator ----
 * Every rank calls each of them, in the same order, after its own
 * tfidf_commit; a rank that cannot serve still takes part.  Its status rides in
 * the first collective of the call (a header ahead of its top-k keys, or the
 * count row of a variable-length gather), so no rank is left waiting:
 *   commits and GLOBAL searches: every rank returns the failing rank's error
 *     together (TFIDF_E_STATE for an index not committed, or re-committed since
 *     the last tfidf_dist_global_commit; TFIDF_E_INVALID_ARG when two ranks'
 *     [doc_base, doc_base + num_docs) ranges overlap: merge keys would collide);
 *   SHARD searches: the other ranks' hits are merged without the failing rank
 *     (Leader.start skips a failed worker, Leader.java:67-69): TFIDF_OK, the
 *     skipped ranks in tfidf_dist_last_failed and a tfidf_last_error() message
 *     naming them; only when no rank can serve is the error returned.  A rank
 *     whose index was re-committed after tfidf_dist_shard_commit is skipped.
 * A query that does not parse
 * (TFIDF_E_QUERY_SYNTAX / _UNSUPPORTED_QUERY) fails on every rank alike before
 * any collective (the reference's Worker answers [] and its Leader merges
 * nothing, Worker.java:182-185).
 *
 * tfidf_dist_global_commit: GLOBAL statistics (term ownership); the shards
 *   whose commits hashed long / non-ASCII terms with different seeds first agree
 *   on the highest attempt (the others re-commit under it).  Outputs may be
 *   NULL (n_vocab = distinct terms over all shards: one more collective).
 * tfidf_dist_search: k >= 1 top-k, or k == 0 every hit, with global doc ids
 *   (doc_base = this shard's first global id); *n_out = hits; TFIDF_E_BUFFER if
 *   they exceed cap (the first cap are written; the whole list stays readable
 *   through tfidf_dist_last_hits, no collective).
 * tfidf_dist_search_batch: n_q queries, 1 <= k <= 1024, outputs n_q x k.
 * tfidf_dist_shard_commit: SHARD mode name table (every rank's document keys,
 *   sorted by String.compareTo, de-duplicated); *n_names may be NULL.
 * tfidf_dist_shard_search: Leader.start over the ranks: *n_out distinct names,
 *   *n_bytes of name text; read them with tfidf_dist_last_names. */
int tfidf_dist_global_commit(tfidf_index *ix, tfidf_comm *c, uint64_t *n_vocab, uint64_t *doc_count,
                             uint64_t *sum_ttf);
int tfidf_dist_search(tfidf_index *ix, tfidf_comm *c, uint64_t doc_base, const uint8_t *q, uint64_t q_len,
                      uint32_t k, uint64_t *doc_ids, float *scores, uint64_t cap, uint64_t *n_out);
int tfidf_dist_search_batch(tfidf_index *ix, tfidf_comm *c, uint64_t doc_base, const uint8_t *q_utf8,
                            const uint64_t *q_offsets, uint32_t n_q, uint32_t k, uint64_t *doc_ids, float *scores,
                            uint32_t *counts);
int tfidf_dist_shard_commit(tfidf_index *ix, tfidf_comm *c, uint64_t *n_names);
int tfidf_dist_shard_search(tfidf_index *ix, tfidf_comm *c, const uint8_t *q, uint64_t q_len, uint64_t *n_out,
                            uint64_t *n_bytes);
/* Results of the communicator's last search (local copies, no collective). */
int tfidf_dist_last_hits(const tfidf_comm *c, uint64_t *doc_ids, float *scores, uint64_t cap, uint64_t *n_out);
/* Ranks skipped by the last SHARD search (bit r = rank r; 0 = every rank answered). */
int tfidf_dist_last_failed(const tfidf_comm *c, uint64_t *rank_mask);
/* names concatenated into buf (cap bytes), offsets[n + 1], scores[n] (double sums) */
int tfidf_dist_last_names(const tfidf_comm *c, uint8_t *buf, uint64_t cap, uint64_t *offsets, double *scores,
                          uint64_t n_cap, uint64_t *n_out, uint64_t *n_bytes);

/* ---- process model (1): one process, one shard per GPU of a device list ----
 * cfg applies to every shard (cfg->device is ignored; cfg->stats_mode selects
 * GLOBAL or SHARD results).  tfidf_node_create: the devices of device_mask (bit
 * i = HIP device i).  tfidf_node_create_devices: an explicit list (a repeated
 * device forces the in-process transport). */
#define TFIDF_NODE_INPROC 1u   /* flags: in-process host transport instead of RCCL */
int tfidf_node_create(const tfidf_config *cfg, uint64_t device_mask, tfidf_node **out);
int tfidf_node_create_devices(const tfidf_config *cfg, const int32_t *devices, uint32_t n_devices, uint32_t flags,
                              tfidf_node **out);
int tfidf_node_destroy(tfidf_node *n);
/* shard i's index (owned by the node): per-shard calls such as tfidf_add_docs_device.
 * A shard changed or committed through this handle needs tfidf_node_commit
 * again: until then GLOBAL searches fail (TFIDF_E_STATE) and SHARD searches
 * skip that shard. */
int tfidf_node_shard(tfidf_node *n, uint32_t i, tfidf_index **ix, uint32_t *n_shards);
/* Documents go to one shard (shard >= 0: the caller routes, as Leader.upload
 * picks a worker, Leader.java:153-207) or are split contiguously over the shards
 * (shard == -1).  Replace-by-key applies within a shard. */
int tfidf_node_add_docs(tfidf_node *n, int32_t shard, const uint8_t *utf8, const uint64_t *offsets, uint64_t n_docs,
                        const uint8_t *keys, const uint64_t *key_offsets);
/* Commits every shard (in parallel), then GLOBAL statistics or the SHARD name table. */
int tfidf_node_commit(tfidf_node *n);
/* GLOBAL mode; same results as tfidf_dist_search / _batch (global doc ids). */
int tfidf_node_search(tfidf_node *n, const uint8_t *q, uint64_t q_len, uint32_t k, uint64_t *doc_ids, float *scores,
                      uint64_t cap, uint64_t *n_out);
int tfidf_node_search_batch(tfidf_node *n, const uint8_t *q_utf8, const uint64_t *q_offsets, uint32_t n_q, uint32_t k,
                            uint64_t *doc_ids, float *scores, uint32_t *counts);
/* SHARD mode (Leader.start): name-ordered {name: double} of the merged hits.
 * A shard that cannot serve is skipped (Leader.java:67-69): TFIDF_OK with the
 * other shards' merged hits, tfidf_node_last_failed names the skipped shards
 * and tfidf_last_error() their reasons. */
int tfidf_node_search_names(tfidf_node *n, const uint8_t *q, uint64_t q_len, uint8_t *buf, uint64_t cap,
                            uint64_t *offsets, double *scores, uint64_t n_cap, uint64_t *n_out, uint64_t *n_bytes);
/* Shards skipped by the last tfidf_node_search_names (bit g = shard g). */
int tfidf_node_last_failed(const tfidf_node *n, uint64_t *shard_mask);
/* Global doc id -> its document key (Worker.java:235-236, across shards). */
int tfidf_node_doc_key(tfidf_node *n, uint64_t doc, uint8_t *buf, uint64_t cap, uint64_t *n_out);
typedef struct tfidf_node_stats {
  uint64_t n_shards;
  uint64_t num_docs;      /* all shards */
  uint64_t doc_count;     /* node statistics in force (GLOBAL: exchanged; SHARD: sum of the shards') */
  uint64_t sum_ttf;
  uint64_t num_terms;     /* distinct terms over all shards (GLOBAL mode), else 0 */
  uint64_t transport;     /* TFIDF_TRANSPORT_RCCL or _INPROC */
} tfidf_node_stats;
int tfidf_node_stats_get(const tfidf_node *n, tfidf_node_stats *out);

/* ---- synthetic corpus (bench/test input generator, device side) ----
 * Zipf(s) over V ranks, rank r -> bijective base-26 word of
 * (r + 18278), doc lengths uniform in [len_min, len_max], ' ' separators and
 * '\n' after every 16th token and after the last.  cdf = double[V] (host). */
int tfidf_synth_corpus(int device, uint64_t seed, uint64_t n_docs, uint64_t doc_base, const double *cdf,
                       uint32_t V, uint32_t len_min, uint32_t len_max, void **d_text, void **d_offsets,
                       uint64_t *total_bytes);
int tfidf_device_free(int device, void *d_ptr);
/* Synchronous copy through the library's own HIP runtime (test/bench helper:
 * a process may hold a second HIP runtime, e.g. PyTorch's bundled one, whose
 * handles do not see the library's allocations).  kind 1 = host -> device,
 * 2 = device -> host. */
int tfidf_device_copy(int device, void *dst, const void *src, uint64_t bytes, int kind);

#ifdef __cplusplus
}
#endif
#endif /* TFIDF_H */
