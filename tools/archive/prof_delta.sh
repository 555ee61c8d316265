#!/bin/bash
# PMC counters of the tokenize kernel with TFIDF_DEBUG_STOP=$1 and =$2 (200k docs).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_delta; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for s in $1 $2; do
 for g in 1 2; do
  if [ $g = 1 ]; then C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"; else C="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN"; fi
  TFIDF_DEBUG_STOP=$s timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex tokenize_wave -d $O/s${s}g$g -o p --output-format csv -- python3 $R/bench.py --docs 200000 --steps 1 --warmup 0 --no-queries --cpu-sample 0 > $O/s${s}g$g.log 2>&1 || exit 2
 done
done
python3 - $O $1 $2 <<'PY'
import csv, collections, glob, sys
O, a, b = sys.argv[1:]
def agg(s):
    d = collections.defaultdict(float)
    for f in glob.glob("%s/s%sg*/*counter_collection.csv" % (O, s)):
        for r in csv.DictReader(open(f)):
            d[r["Counter_Name"]] += float(r["Counter_Value"])
    return d
A, B = agg(a), agg(b)
for k in sorted(A):
    print("%-24s stop%s=%.3e stop%s=%.3e delta/doc=%.1f" % (k, a, A[k], b, B[k], (B[k] - A[k]) / 200000))
PY
