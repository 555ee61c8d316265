#!/bin/bash
# Query-path kernel timings: rocprofv3 kernel-trace summary of a bench run with queries.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/kt_queries; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-e2e --cpu-sample 0 ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "kt failed"; tail -5 $O/bench.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-40s calls=%5s avg_ms=%8.4f total_ms=%9.3f" % (r["Name"].split("(")[0][-40:], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
