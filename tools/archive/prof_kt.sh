#!/bin/bash
# rocprofv3 kernel-trace summary of one bench command (GPU box).
# Usage: TAG=name ARGS="--steps 1 ..." bash tools/archive/prof_kt.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/kt_${TAG:-q}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py ${ARGS:-} > $O/bench.log 2>&1 || { echo "kt failed"; tail -5 $O/bench.log; exit 1; }
f=$(find $O -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:25]:
    print("%-60s %6s %10.3f ms avg %9.4f ms" % (r["Name"].split("(")[0][:60], r["Calls"], float(r["TotalDurationNs"]) / 1e6,
                                               float(r["AverageNs"]) / 1e6))
PY
