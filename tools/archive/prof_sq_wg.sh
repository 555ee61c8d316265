#!/bin/bash
# SQ counters per document: wave tokenizer vs workgroup tokenizer (TFIDF_TOK_WG), 200 k cfg-2 docs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/sqwg; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_BUSY_CYCLES"
for k in wave wg; do
 for g in 1 2; do
  if [ $g = 1 ]; then C=$G1; else C=$G2; fi
  if [ $k = wg ]; then export TFIDF_TOK_WG=1; else unset TFIDF_TOK_WG; fi
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "tokenize_w" -d $O/${k}g$g -o p --output-format csv -- python3 $R/bench.py --docs 200000 --steps 1 --warmup 0 --no-queries --no-e2e --cpu-sample 0 > $O/${k}g$g.log 2>&1 || { echo "pmc $k g=$g failed"; tail -3 $O/${k}g$g.log; exit 2; }
 done
done
unset TFIDF_TOK_WG
python3 - $O <<'PY'
import csv, collections, glob, sys
O = sys.argv[1]
for k in ("wave", "wg"):
    d = collections.defaultdict(float); n = collections.defaultdict(set)
    for f in glob.glob("%s/%sg*/**/*counter_collection.csv" % (O, k), recursive=True):
        for r in csv.DictReader(open(f)):
            d[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(k, {c: round(v / max(len(n[c]), 1) / 200000, 1) for c, v in sorted(d.items())})
PY
