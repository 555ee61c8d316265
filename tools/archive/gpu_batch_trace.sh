#!/bin/bash
# Kernel trace of the 10 k-query batch (tools/time_batch_host.py): per-kernel
# durations of the unit scorers and the merge.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_batch -o batch --output-format csv -- python3 $R/tools/time_batch_host.py > $R/gpurun_out/prof_batch.log 2>&1 || { echo "trace failed"; tail -3 $R/gpurun_out/prof_batch.log; exit 1; }
f=$(find $R/gpurun_out/prof_batch -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print("%-60s calls %5s avg %.3f ms total %.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
