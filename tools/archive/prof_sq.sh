#!/bin/bash
# SQ counters per dispatch of the tokenizer kernels for one small build (GPU box).
# Usage: LIB=path TOK=lf|wave bash tools/archive/prof_sq.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sq_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/tools/ab_build.py ${LIB:-$R/tf-idf-distributed-system_amd/lib/libtfidf.so}"
export AB_CORPUS=${AB_CORPUS:-docs=200000}
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "k_tokenize" -d $O/p1 -o p1 --output-format csv -- $CMD > $O/p1.log 2>&1 || { echo "p1 failed"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_FLAT --kernel-include-regex "k_tokenize" -d $O/p2 -o p2 --output-format csv -- $CMD > $O/p2.log 2>&1 || { echo "p2 failed"; tail -5 $O/p2.log; exit 2; }
python3 - $O <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(float)
waves = 0
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])] += float(r["Counter_Value"])
names = sorted(set(k for k, _ in acc))
for n in names:
    w = acc.get((n, "SQ_WAVES"), 0) or 1
    print(n, {c: round(v / w, 1) for (k, c), v in sorted(acc.items()) if k == n})
PY
