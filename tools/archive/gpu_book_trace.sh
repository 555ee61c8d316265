#!/bin/bash
# Kernel traces of the 300-book shapes (ASCII, and one non-ASCII word per ~2 KB).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for shape in book bookuni; do
  A="--steps 5 --warmup 2 --docs 300 --len-min 80000 --len-max 120000 --no-queries --no-e2e --cpu-sample 0"
  [ $shape = bookuni ] && A="$A --unicode-every 2048"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$shape -o $shape --output-format csv -- python3 $R/bench.py $A > $R/gpurun_out/prof_$shape.log 2>&1 || { echo "$shape trace failed"; tail -3 $R/gpurun_out/prof_$shape.log; exit 1; }
  f=$(find $R/gpurun_out/prof_$shape -name "*kernel_stats.csv" | head -1)
  echo "== $shape"
  python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:12]:
    print("%-60s calls %5s avg %.3f ms total %.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
done
