#!/bin/bash
# PMC passes on the index-build kernels (reduced 200k-doc run), one pass per counter group.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_${TAG:-x}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --docs 200000 --steps 1 --warmup 0 --no-queries --cpu-sample 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B > $O/kt.log 2>&1 || exit 1
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "tokenize|scatter|df_partial" -d $O/p$i -o p$i --output-format csv -- $B > $O/p$i.log 2>&1 || exit 2
done
python3 - $O <<'PY'
import csv, collections, glob, sys
O = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(O + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: "%.3g" % v for c, v in sorted(d.items())})
PY
cat $O/kt/kt_kernel_stats.csv | cut -d, -f1-4
