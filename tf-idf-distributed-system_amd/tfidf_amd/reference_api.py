"""Host-side mirror of the reference's hot-path interface, over the GPU engine.

Java cannot be built in this image, so the reference's own host classes are
mirrored here with the same names, argument meaning and error behaviour, each
method citing the reference code it stands in for (paths relative to
TF-IDF-System-Core/src/main/java/).  INTEGRATION.md shows the JNI binding a
maintainer adds to the Java classes themselves.

  Worker  <- me/zookeeper/leader_election/worker/Worker.java
  Leader  <- me/zookeeper/leader_election/leader/Leader.java
  DocumentScoreInfo JSON <- Document_and_Data/DocumentScoreInfo.java:11-31,
                            Document_and_Data/Document.java:6-53
"""
import os

from . import _lib as L
from .engine import ShardIndex, leader_merge


def extract_text(data: bytes) -> bytes:
    """Stand-in for the reference's Tika fallback (AutoDetectParser +
    BodyContentHandler, Worker.java:201-211) on a file that is not valid
    UTF-8: plain text in a single-byte Western encoding is decoded as
    windows-1252 (bytes it leaves undefined as Latin-1) and re-encoded as
    UTF-8.  Tika's own charset detection and its parsers for binary formats
    (PDF, Office) are not rebuilt: parity unpinned."""
    out = []
    for b in data:
        try:
            out.append(bytes([b]).decode("cp1252"))
        except UnicodeDecodeError:
            out.append(chr(b))
    return "".join(out).encode("utf-8")


def document_score_info(name: str, score: float):
    """Jackson form of DocumentScoreInfo: {"document": {"name": ...}, "score": double}."""
    return {"document": {"name": name}, "score": float(score)}


class Worker:
    """Worker.java:42-242 — one shard: builds its index at init, answers
    /worker/process with every hit of its shard-local BM25 ranking."""

    def __init__(self, documents_path=None, index_path=None, device=0, vocab_capacity_log2=18):
        # @Value("${mydocument.path}") / @Value("${lucene.index.path}") (Worker.java:48-52)
        self.DOCUMENTS_PATH = documents_path
        self.INDEX_PATH = index_path
        self.index = ShardIndex(device=device, vocab_capacity_log2=vocab_capacity_log2)
        self._committed = False

    INDEX_FILE = "tfidf.idx"

    def _index_file(self):
        return os.path.join(self.INDEX_PATH, self.INDEX_FILE) if self.INDEX_PATH else None

    # Worker.java:57-94 @PostConstruct init: open the index directory
    # (IndexWriterConfig default OpenMode CREATE_OR_APPEND: a saved index is
    # reopened), walk the documents directory skipping the index directory,
    # addDocToIndex per regular file (replacing by relative path), commit.
    def init(self):
        idx_file = self._index_file()
        if idx_file and os.path.isfile(idx_file):
            self.index.load(idx_file)
        docs_path = os.path.normpath(self.DOCUMENTS_PATH)
        if not os.path.isdir(docs_path):
            if idx_file and os.path.isfile(idx_file):
                self.commit()
            return
        idx_path = os.path.normpath(self.INDEX_PATH) if self.INDEX_PATH else None
        paths = []
        # Files.walk order is file-system dependent; sorted depth-first here so
        # document ids (tie-break order) are reproducible.
        for root, dirs, files in os.walk(docs_path):
            dirs.sort()
            if idx_path and os.path.normpath(root).startswith(idx_path):
                continue
            dirs[:] = [d for d in dirs if not (idx_path and os.path.join(root, d).startswith(idx_path))]
            for f in sorted(files):
                paths.append(os.path.join(root, f))
        keys, texts = [], []
        for p in paths:
            try:
                k, t = self._read(p)
            except OSError:
                continue                      # Worker.java:83-85: log and skip
            keys.append(k)
            texts.append(t)
        self.index.add_documents(texts, keys)
        self.commit()

    def _read(self, path):
        base = os.path.normpath(self.DOCUMENTS_PATH)
        absp = os.path.normpath(path)
        # Worker.java:191-195: RELATIVE path is the document key
        rel = os.path.relpath(absp, base) if absp.startswith(base + os.sep) else os.path.basename(absp)
        with open(absp, "rb") as f:
            data = f.read()
        try:
            data.decode("utf-8")              # Files.readString: strict UTF-8
        except UnicodeDecodeError:
            data = extract_text(data)         # MalformedInputException -> Tika (Worker.java:199-211)
        return rel.encode(), data

    # Worker.java:190-220 addDocToIndex (updateDocument by Term("path", rel))
    def add_doc_to_index(self, path):
        k, t = self._read(path)
        self.index.add_documents([t], [k])

    # Worker.java:88,138 indexWriter.commit(): the index becomes durable
    def commit(self):
        self.index.commit()
        self._committed = True
        idx_file = self._index_file()
        if idx_file:
            os.makedirs(self.INDEX_PATH, exist_ok=True)
            self.index.save(idx_file)

    # Worker.java:125-146 upload: copy the file, then add + commit under the writer lock
    def upload(self, filename, data: bytes):
        if not data:
            return 400, "Empty file"
        try:
            dest = os.path.normpath(os.path.join(self.DOCUMENTS_PATH, filename))
            with open(dest, "wb") as f:
                f.write(data)
            self.add_doc_to_index(dest)
            self.commit()
            return 200, "Uploaded"
        except Exception as e:                # Worker.java:142-145
            return 500, "Upload failed: %s" % e

    # Worker.java:147-172 /worker/index-size (bytes held by the index)
    def get_index_size(self):
        return int(self.index.stats()["device_bytes"]) if self._committed else 0

    # Worker.java:222-241 searchIndex: every hit, score desc / doc asc
    def search_index(self, query: str):
        # one reader per request: hits and their stored paths from the same commit (:223, :234-238)
        with self.index.reader() as rd:
            hits = rd.search(query.encode(), 0)
            return [document_score_info(rd.doc_key(d).decode(), s) for d, s in hits]

    # Worker.java:175-186 /worker/process: any exception -> empty list
    def process_documents(self, search_query: str):
        try:
            return self.search_index(search_query)
        except Exception:
            return []

    def close(self):
        self.index.close()


class Leader:
    """Leader.java:39-92 /leader/start: fan the query out to every worker
    (sequentially; failed workers are skipped), sum scores per document name
    in double, return the map ordered by name."""

    def __init__(self, workers):
        self.workers = workers                # ServiceRegistry.getAllServiceAddresses()

    def start(self, search_query: str):
        if not self.workers:
            return {}                         # Leader.java:45-48
        responses = []
        for w in self.workers:
            try:
                resp = w.process_documents(search_query)
            except Exception:
                continue                      # Leader.java:67-69
            if resp is None:
                continue
            responses.append([(r["document"]["name"].encode(), r["score"]) for r in resp])
        merged = leader_merge(responses)      # Leader.java:73-88
        return {name.decode(): score for name, score in merged}


__all__ = ["Worker", "Leader", "document_score_info", "L"]
