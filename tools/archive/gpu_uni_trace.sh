#!/bin/bash
# Kernel trace of cfg 2 with a fraction of non-ASCII documents (UF, default 1.0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
UF=${UF:-1.0}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_uf -o uf --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-queries --no-e2e --cpu-sample 0 --unicode-frac $UF > $R/gpurun_out/prof_uf.log 2>&1 || { echo "trace failed"; tail -3 $R/gpurun_out/prof_uf.log; exit 1; }
f=$(find $R/gpurun_out/prof_uf -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print("%-60s calls %5s avg %.3f ms total %.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
