#!/bin/bash
# SQ counters + kernel trace of the query-unit batch kernel (cfg-4 batch over the cfg-2 index).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sq_units
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ONLY_UNITS=1
CMD="python3 $R/tools/batch_units.py"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $CMD > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "k_score_.*units" -d $O/p1 -o p1 --output-format csv -- $CMD > $O/p1.log 2>&1 || { echo "p1 failed"; tail -5 $O/p1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_BRANCH --kernel-include-regex "k_score_.*units" -d $O/p2 -o p2 --output-format csv -- $CMD > $O/p2.log 2>&1 || { echo "p2 failed"; tail -5 $O/p2.log; exit 2; }
python3 - $O <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
for f in glob.glob(d + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-40s calls=%5s avg_ms=%8.4f" % (r["Name"].split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e6))
acc = collections.defaultdict(float)
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])] += float(r["Counter_Value"])
for n in sorted(set(k for k, _ in acc)):
    print(n, {c: "%.4g" % v for (kn, c), v in sorted(acc.items()) if kn == n})
PY
