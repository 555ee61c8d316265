#!/bin/bash
# kernel-trace summary of a short build-only bench (ARGS passed to bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${TAG:-kt_build}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-queries --no-e2e --cpu-sample 0 ${ARGS:-} > $O/log 2>&1 || { echo "kt failed"; tail -5 $O/log; exit 1; }
python3 - $O <<'P'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1]+'/kt_kernel_stats.csv')))
for r in rows[:24]: print("%-60s %6s %10.1f us" % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
P
