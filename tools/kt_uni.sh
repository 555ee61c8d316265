#!/bin/bash
# Kernel trace of one cfg-2 build with every document non-ASCII: the ASCII
# pass, the UNI pass and the Unicode wave path separately (round 5).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/kt_uni; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 --no-e2e --unicode-frac ${FRAC:-1.0} > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
f = glob.glob(O + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "tokenize" in r["Kernel_Name"]:
        d[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    v = sorted(v); print("%-60s n=%d median %.3f ms" % (k, len(v), v[len(v) // 2]))
PY
