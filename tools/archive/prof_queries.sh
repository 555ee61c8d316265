#!/bin/bash
# PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and SQ counters of the query kernels in the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/prof_q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-e2e"
RX="k_score|k_merge|k_hits"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --kernel-include-regex "$RX" -d $O/kt -o kt --output-format csv -- $CMD > $O/kt.log 2>&1 || { echo kt failed; tail -3 $O/kt.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d $O/fetch -o fetch --output-format csv -- $CMD > $O/fetch.log 2>&1 || { echo fetch failed; tail -3 $O/fetch.log; exit 2; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d $O/write -o write --output-format csv -- $CMD > $O/write.log 2>&1 || { echo write failed; tail -3 $O/write.log; exit 3; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-include-regex "$RX" -d $O/sq -o sq --output-format csv -- $CMD > $O/sq.log 2>&1 || { echo sq failed; tail -3 $O/sq.log; exit 4; }
python3 - $O <<'P'
import csv, glob, sys, collections
O = sys.argv[1]
def agg(pat):
    d = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for f in glob.glob(O + pat, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1]
            d[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    return d, n
for pat in ("/fetch/**/*counter_collection.csv", "/write/**/*counter_collection.csv", "/sq/**/*counter_collection.csv"):
    d, n = agg(pat)
    for k in sorted(d):
        print("%-34s dispatches %5d  " % (k[:34], len(n[k])) + "  ".join("%s=%.3g" % (c, v / len(n[k])) for c, v in sorted(d[k].items())))
P
