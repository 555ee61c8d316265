#!/bin/bash
# Instruction-cache counters of the wave tokenizer (one PMC pass, bounded).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_icache
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH --kernel-include-regex "tokenize_wave|scatter|df_partial" -d $O/ic -o ic --output-format csv -- python3 $R/bench.py --docs 200000 --steps 1 --warmup 0 --no-queries --cpu-sample 0 --no-e2e > $O/ic.log 2>&1 || { echo "icache pass failed"; tail -5 $O/ic.log; exit 2; }
python3 - $O <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/ic/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        d[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])] += float(r["Counter_Value"])
for k in sorted(d):
    print("%-50s %-28s %.4g" % (k[0][-50:], k[1], d[k]))
PY
