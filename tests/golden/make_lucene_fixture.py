#!/usr/bin/env python3
"""Decode the reference's committed Lucene 9.8.0 index into a JSON golden fixture.

This is the ONLY artefact in the reference that pins tokenisation / TF / DF /
norms / collection statistics produced by real Lucene.
The script reads the index files as plain bytes (no code from the reference is
executed or copied) and writes ``tests/golden/lucene_sample8.json``.  The JSON
is committed; the script is re-runnable only where ``/root/reference`` exists.

Decoded structures (Lucene 9.8.0 on-disk formats, restated from the public
Lucene90 codec specification):

* ``_6.nvm`` / ``_6.nvd``  Lucene90NormsFormat: per-field meta record
  (field number, docsWithField, numDocsWithValue, bytesPerNorm, normsOffset),
  then one norm byte per doc in ``.nvd``.
* ``_6_Lucene90_0.tmd``    BlockTree terms meta: per field numTerms,
  sumTotalTermFreq, sumDocFreq, docCount.
* ``_6_Lucene90_0.tim``    BlockTree leaf block: suffix bytes, suffix lengths,
  per-term stats (docFreq, totalTermFreq with singleton run-length coding).
* ``_6_Lucene90_0.doc``    Lucene90 postings: for docFreq < 128 every posting
  is a VInt ``docDelta << 1 | (freq == 1)`` followed by VInt freq when != 1.

Provenance offsets (bytes) are recorded in the fixture.
"""
import json
import os
import struct
import sys

REF = "/root/reference/TF-IDF-System-Core/src/main/resources"
IDX = os.path.join(REF, "documents", ".luceneIndex")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lucene_sample8.json")

CODEC_MAGIC = 0x3FD76C17


class Reader:
    def __init__(self, data, pos=0):
        self.d = data
        self.p = pos

    def byte(self):
        b = self.d[self.p]
        self.p += 1
        return b

    # Codec headers are big-endian (CodecUtil.writeBEInt); since Lucene 9.0
    # every other fixed-width int/long/short in DataOutput is little-endian.
    def be_int(self):
        v = struct.unpack(">i", self.d[self.p:self.p + 4])[0]
        self.p += 4
        return v

    def le_int(self):
        v = struct.unpack("<i", self.d[self.p:self.p + 4])[0]
        self.p += 4
        return v

    def le_long(self):
        v = struct.unpack("<q", self.d[self.p:self.p + 8])[0]
        self.p += 8
        return v

    def le_short(self):
        v = struct.unpack("<h", self.d[self.p:self.p + 2])[0]
        self.p += 2
        return v

    def vint(self):
        shift = 0
        v = 0
        while True:
            b = self.byte()
            v |= (b & 0x7F) << shift
            if b < 0x80:
                return v
            shift += 7

    vlong = vint

    def raw(self, n):
        s = self.d[self.p:self.p + n]
        self.p += n
        return s

    def string(self):
        n = self.vint()
        return self.raw(n).decode("utf-8")

    def index_header(self):
        """CodecUtil.checkIndexHeader: magic, codec name, version, id[16], suffix."""
        magic = self.be_int() & 0xFFFFFFFF
        assert magic == CODEC_MAGIC, hex(magic)
        name = self.string()
        version = self.be_int()
        self.raw(16)
        suffix_len = self.byte()
        suffix = self.raw(suffix_len).decode()
        return name, version, suffix


def read(path):
    with open(path, "rb") as f:
        return f.read()


def decode_norms():
    meta = Reader(read(os.path.join(IDX, "_6.nvm")))
    meta.index_header()
    field = meta.le_int()
    docs_with_field_offset = meta.le_long()
    meta.le_long()      # docsWithFieldLength
    meta.le_short()     # jumpTableEntryCount
    meta.byte()         # denseRankPower
    num_docs_with_value = meta.le_int()
    bytes_per_norm = meta.byte()
    norms_offset = meta.le_long()
    assert docs_with_field_offset == -1 and bytes_per_norm == 1
    data = read(os.path.join(IDX, "_6.nvd"))
    norms = list(data[norms_offset:norms_offset + num_docs_with_value])
    return field, norms, norms_offset


def decode_field_stats():
    r = Reader(read(os.path.join(IDX, "_6_Lucene90_0.tmd")))
    r.index_header()                       # BlockTreeTermsMeta
    r.index_header()                       # Lucene90PostingsWriterTerms
    block_size = r.vint()
    assert block_size == 128
    num_fields = r.vint()
    out = {}
    for _ in range(num_fields):
        start = r.p
        field = r.vint()
        num_terms = r.vlong()
        root_len = r.vint()
        r.raw(root_len)
        # index options >= DOCS_AND_FREQS for "contents"; "path" is DOCS only
        # (StringField) and omits sumTotalTermFreq.
        if field == 1:
            sum_ttf = r.vlong()
            sum_df = r.vlong()
            doc_count = r.vint()
            min_term = r.raw(r.vint()).decode()
            max_term = r.raw(r.vint()).decode()
            out["contents"] = dict(field=field, numTerms=num_terms,
                                   sumTotalTermFreq=sum_ttf, sumDocFreq=sum_df,
                                   docCount=doc_count, minTerm=min_term,
                                   maxTerm=max_term, tmd_offset=start)
            break
        raise RuntimeError("unexpected field order in .tmd")
    return out["contents"]


def decode_terms(num_terms):
    r = Reader(read(os.path.join(IDX, "_6_Lucene90_0.tim")))
    r.index_header()
    block_start = r.p
    code = r.vint()
    ent_count = code >> 1
    assert ent_count == num_terms
    token = r.vlong()
    suffix_bytes = token >> 3
    is_leaf = bool(token & 0x04)
    compression = token & 0x03
    assert is_leaf and compression == 0
    suffixes = r.raw(suffix_bytes)
    tok2 = r.vint()
    n_len = tok2 >> 1
    all_equal = tok2 & 1
    assert not all_equal and n_len == ent_count
    lens = list(r.raw(n_len))
    terms = []
    p = 0
    for ln in lens:
        terms.append(suffixes[p:p + ln].decode())
        p += ln
    stats_len = r.vint()
    s = Reader(r.raw(stats_len))
    stats = []
    singleton_run = 0
    for _ in terms:
        if singleton_run > 0:
            singleton_run -= 1
            stats.append((1, 1))
            continue
        tok = s.vint()
        if tok & 1:
            singleton_run = tok >> 1
            stats.append((1, 1))
        else:
            df = tok >> 1
            ttf = df + s.vlong()
            stats.append((df, ttf))
    return terms, stats, block_start


def decode_postings(terms, stats):
    r = Reader(read(os.path.join(IDX, "_6_Lucene90_0.doc")))
    r.index_header()
    start = r.p
    postings = {}
    for term, (df, ttf) in zip(terms, stats):
        assert df > 1 and df < 128, "singleton/pfor blocks not present in fixture"
        doc = 0
        plist = []
        for _ in range(df):
            code = r.vint()
            doc += code >> 1
            freq = 1 if (code & 1) else r.vint()
            plist.append([doc, freq])
        assert sum(f for _, f in plist) == ttf, term
        postings[term] = plist
    return postings, start, r.p


def main():
    if not os.path.isdir(IDX):
        print("reference index not present; fixture is committed", file=sys.stderr)
        return 1
    field, norms, norms_off = decode_norms()
    fstats = decode_field_stats()
    terms, stats, tim_off = decode_terms(fstats["numTerms"])
    postings, doc_off, doc_end = decode_postings(terms, stats)
    names = ["file.txt"] + ["file%d.txt" % i for i in range(2, 9)]
    docs = []
    for n in names:
        with open(os.path.join(REF, "documents", n), "rb") as f:
            docs.append({"name": n, "text": f.read().decode("ascii")})
    lengths = [0] * len(norms)
    for plist in postings.values():
        for d, f in plist:
            lengths[d] += f
    fixture = {
        "provenance": {
            "source": "reference TF-IDF-System-Core/src/main/resources/documents/.luceneIndex (segment _6, lucene.version 9.8.0)",
            "generator": "tests/golden/make_lucene_fixture.py",
            "offsets": {"nvd_norms": norms_off, "tim_block": tim_off,
                        "doc_postings": [doc_off, doc_end],
                        "tmd_field": fstats["tmd_offset"]},
            "note": "docs 0-7 = file.txt, file2.txt..file8.txt in Files.walk order; "
                    "docs 8-20 are Lucene's own index files indexed with no tokens (norm 0)",
        },
        "max_doc": len(norms),
        "docs": docs,
        "field_stats": {k: fstats[k] for k in ("numTerms", "sumTotalTermFreq", "sumDocFreq", "docCount", "minTerm", "maxTerm")},
        "norms": norms,
        "doc_lengths_from_postings": lengths,
        "terms": [{"term": t, "df": df, "ttf": ttf, "postings": postings[t]}
                  for t, (df, ttf) in zip(terms, stats)],
    }
    with open(OUT, "w") as f:
        json.dump(fixture, f, indent=1)
        f.write("\n")
    print("wrote", OUT)
    return 0


if __name__ == "__main__":
    sys.exit(main())
