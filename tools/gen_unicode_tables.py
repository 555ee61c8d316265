#!/usr/bin/env python3
"""Generate the Unicode property tables of the general (Unicode) tokenizer.

Run here (needs ICU 70's libicuuc, present in this image); the outputs are
committed, so nothing at build or run time needs ICU:

  tf-idf-distributed-system_amd/csrc/unicode_tables.h  two-stage tables (product)
  oracle/unicode_props.h                                range / pair lists (oracle)

What they restate ("Unicode"):
  * Lucene 9.8.0 StandardTokenizerImpl is a JFlex scanner generated with
    `%unicode 9.0`: character classes are the Unicode 9.0 Word_Break values,
    plus Script=Han / Script=Hiragana / Line_Break=Complex_Context and the
    emoji / Regional_Indicator classes of its grammar.  Property values come
    from ICU 70 (Unicode 14) restricted to code points ASSIGNED in Unicode 9.0
    (u_charAge <= 9.0); later code points are class Other.  Values of 9.0-era
    code points that changed between 9.0 and 14 (emoji E_Base/E_Modifier/
    Glue_After_Zwj were folded into Extend / Extended_Pictographic in 11.0)
    are mapped as the grammar uses them (E_Modifier -> extender).
  * LowerCaseFilter calls Character.toLowerCase(int) of the reference's JDK 17
    (Dockerfile:1, openjdk:17 = Unicode 13.0): the simple lowercase mapping,
    taken from Python 3.10's unicodedata (also Unicode 13.0): chr(c).lower()
    when that is one code point; U+0130 (whose full mapping is two code points)
    maps to U+0069 as in UnicodeData.txt.
"""
import ctypes as C
import os
import sys
import unicodedata

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ICU = C.CDLL("libicuuc.so.70")
V = "_70"
u_charAge = getattr(ICU, "u_charAge" + V)
u_charAge.argtypes = [C.c_int32, C.POINTER(C.c_uint8)]
u_getIntPropertyValue = getattr(ICU, "u_getIntPropertyValue" + V)
u_getIntPropertyValue.argtypes = [C.c_int32, C.c_int]
u_getIntPropertyValue.restype = C.c_int32
u_hasBinaryProperty = getattr(ICU, "u_hasBinaryProperty" + V)
u_hasBinaryProperty.argtypes = [C.c_int32, C.c_int]
u_hasBinaryProperty.restype = C.c_int8

UCHAR_EXTENDED_PICTOGRAPHIC, UCHAR_LINE_BREAK, UCHAR_SCRIPT, UCHAR_WORD_BREAK = 64, 0x1008, 0x100A, 0x1014
(WB_OTHER, WB_ALETTER, WB_FORMAT, WB_KATAKANA, WB_MIDLETTER, WB_MIDNUM, WB_NUMERIC, WB_EXTENDNUMLET, WB_CR,
 WB_EXTEND, WB_LF, WB_MIDNUMLET, WB_NEWLINE, WB_RI, WB_HEBREW, WB_SQ, WB_DQ, WB_EB, WB_EBG, WB_EM, WB_GAZ,
 WB_ZWJ, WB_WSEG) = range(23)
LB_SA, SC_HAN, SC_HIRAGANA = 24, 17, 20

# Tokenizer classes (keep in sync with kUc* in unicode_scan.h and UC_* in oracle/)
CLASSES = ["OTHER", "ALETTER", "HEBREW", "NUMERIC", "KATAKANA", "EXTNUMLET", "MIDLETTER", "MIDNUMLET",
           "MIDNUM", "SQUOTE", "DQUOTE", "EXTEND", "EXTEND_SA", "ZWJ", "SA", "HAN", "HIRAGANA", "RI", "EMOJI"]
K = {n: i for i, n in enumerate(CLASSES)}
MAXCP = 0x110000


def age(cp):
    a = (C.c_uint8 * 4)()
    u_charAge(cp, a)
    return (a[0], a[1])


def klass(cp):
    ag = age(cp)
    if ag == (0, 0) or ag > (9, 0):
        return K["OTHER"]
    if 0xD800 <= cp <= 0xDFFF:
        return K["OTHER"]
    wb = u_getIntPropertyValue(cp, UCHAR_WORD_BREAK)
    lb = u_getIntPropertyValue(cp, UCHAR_LINE_BREAK)
    sc = u_getIntPropertyValue(cp, UCHAR_SCRIPT)
    if wb == WB_ZWJ:
        return K["ZWJ"]
    if wb in (WB_EXTEND, WB_FORMAT, WB_EM) or 0x1F3FB <= cp <= 0x1F3FF:
        return K["EXTEND_SA"] if lb == LB_SA else K["EXTEND"]
    # NumericEx = [\p{WB:Numeric}[\p{Blk:HalfAndFullForms}&&\p{Nd}]]
    if 0xFF00 <= cp <= 0xFFEF and unicodedata.category(chr(cp)) == "Nd":
        return K["NUMERIC"]
    m = {WB_ALETTER: "ALETTER", WB_HEBREW: "HEBREW", WB_NUMERIC: "NUMERIC", WB_KATAKANA: "KATAKANA",
         WB_EXTENDNUMLET: "EXTNUMLET", WB_MIDLETTER: "MIDLETTER", WB_MIDNUMLET: "MIDNUMLET", WB_MIDNUM: "MIDNUM",
         WB_SQ: "SQUOTE", WB_DQ: "DQUOTE", WB_RI: "RI"}
    if wb in m:
        return K[m[wb]]
    if lb == LB_SA:
        return K["SA"]
    if sc == SC_HAN:
        return K["HAN"]
    if sc == SC_HIRAGANA:
        return K["HIRAGANA"]
    if cp >= 0x80 and u_hasBinaryProperty(cp, UCHAR_EXTENDED_PICTOGRAPHIC):
        return K["EMOJI"]
    return K["OTHER"]


def lower(cp):
    if 0xD800 <= cp <= 0xDFFF:
        return cp
    if cp == 0x130:
        return 0x69
    s = chr(cp).lower()
    return ord(s) if len(s) == 1 else cp


def two_stage(values, block=256):
    blocks, index, stage2 = {}, [], []
    for b in range(0, len(values), block):
        t = tuple(values[b:b + block])
        if t not in blocks:
            blocks[t] = len(blocks)
            stage2.extend(t)
        index.append(blocks[t])
    return index, stage2


def carr(name, vals, per=24):
    out = ["#define %s { \\" % name]
    for i in range(0, len(vals), per):
        out.append("  " + ", ".join(str(v) for v in vals[i:i + per]) + ", \\")
    out.append("}")
    return "\n".join(out)


def main():
    cls = [klass(cp) for cp in range(MAXCP)]
    low = [lower(cp) - cp for cp in range(MAXCP)]
    ci, cs = two_stage(cls)
    li, ls = two_stage(low)
    assert max(ci) < 65536 and max(li) < 65536
    hdr = os.path.join(REPO, "tf-idf-distributed-system_amd", "csrc", "unicode_tables.h")
    with open(hdr, "w") as f:
        f.write("// unicode_tables.h — GENERATED by tools/gen_unicode_tables.py (do not edit).\n"
                "// Tokenizer class (kUc*, unicode_scan.h) and simple-lowercase delta per code point,\n"
                "// two-stage tables of 256-code-point blocks.  Sources: ICU 70 properties of code\n"
                "// points assigned in Unicode 9.0 (Lucene 9.8 StandardTokenizerImpl, %unicode 9.0);\n"
                "// JDK 17 Character.toLowerCase (Unicode 13.0).  Initialiser lists only: unicode_scan.h\n"
                "// instantiates them as host and device arrays.\n#pragma once\n")
        f.write("#define TFIDF_UC_CLASS_INDEX_N %d\n#define TFIDF_UC_CLASS_DATA_N %d\n" % (len(ci), len(cs)))
        f.write("#define TFIDF_UC_LOWER_INDEX_N %d\n#define TFIDF_UC_LOWER_DATA_N %d\n" % (len(li), len(ls)))
        f.write(carr("TFIDF_UC_CLASS_INDEX", ci) + "\n")
        f.write(carr("TFIDF_UC_CLASS_DATA", cs, 48) + "\n")
        f.write(carr("TFIDF_UC_LOWER_INDEX", li) + "\n")
        f.write(carr("TFIDF_UC_LOWER_DATA", ls, 16) + "\n")
    # oracle: sorted (first, last, class) ranges of non-OTHER classes, (cp, lower) pairs
    ranges = []
    for cp, k in enumerate(cls):
        if k == 0:
            continue
        if ranges and ranges[-1][1] == cp - 1 and ranges[-1][2] == k:
            ranges[-1][1] = cp
        else:
            ranges.append([cp, cp, k])
    pairs = [(cp, cp + d) for cp, d in enumerate(low) if d]
    ohdr = os.path.join(REPO, "oracle", "unicode_props.h")
    with open(ohdr, "w") as f:
        f.write("/* unicode_props.h — GENERATED by tools/gen_unicode_tables.py (do not edit).\n"
                " * ORACLE data (test infrastructure): Lucene 9.8 StandardTokenizer character classes\n"
                " * (UC_* in tfidf_oracle.c) as sorted code-point ranges, and JDK 17\n"
                " * Character.toLowerCase pairs.  Same sources as the product's tables, other layout. */\n")
        f.write("static const uint32_t uc_ranges[%d][3] = {\n" % len(ranges))
        for a, b, k in ranges:
            f.write("  {0x%X, 0x%X, %d},\n" % (a, b, k))
        f.write("};\n#define UC_NRANGES %d\n" % len(ranges))
        f.write("static const uint32_t uc_lower[%d][2] = {\n" % len(pairs))
        for a, b in pairs:
            f.write("  {0x%X, 0x%X},\n" % (a, b))
        f.write("};\n#define UC_NLOWER %d\n" % len(pairs))
    print("classes: %d blocks, lower: %d blocks, %d ranges, %d lower pairs" %
          (len(cs) // 256, len(ls) // 256, len(ranges), len(pairs)), file=sys.stderr)


if __name__ == "__main__":
    main()
