#!/bin/bash
# XCD-partitioned dictionary bound (tools/calib_xcd.hip): event times per case,
# then one rocprofv3 pass for the L2 hit rate of each case's warm launches.
# Output: gpurun_out/calib_xcd/summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/calib_xcd; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B=$R/tools/bin/calib_xcd
timeout -k 10 120 $B > $O/times.txt 2>&1 || { echo "plain run failed"; cat $O/times.txt; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT TCC_MISS -d $O/p1 -o p --output-format csv -- $B > $O/p1.log 2>&1 || { echo "pmc failed"; tail -3 $O/p1.log; exit 1; }
python3 - $O <<'PY' | tee $O/summary.txt
import csv, glob, sys, collections
O = sys.argv[1]
lines = [l.rstrip("\n") for l in open(O + "/times.txt")]
names = [l.split()[0] for l in lines if l and not l.startswith("#") and not l.startswith("launch")]
vals = collections.defaultdict(dict)
for f in glob.glob(O + "/p1/**/*counter_collection.csv", recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "k_" in r["Kernel_Name"]]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    rank = {d: k for k, d in enumerate(ids)}
    for r in rows:
        d = vals[rank[int(r["Dispatch_Id"])]]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
hit = {}
for k, name in enumerate(names):          # 6 launches per case; the first (cold) is skipped
    h = sum(vals[6 * k + j].get("TCC_HIT", 0) for j in range(1, 6))
    m = sum(vals[6 * k + j].get("TCC_MISS", 0) for j in range(1, 6))
    hit[name] = 100.0 * h / max(h + m, 1)
k = 0
for l in lines:
    if l and not l.startswith("#") and not l.startswith("launch"):
        print("%s %9.1f" % (l, hit.get(l.split()[0], 0)))
    elif l.startswith("launch"):
        print(l + "   L2 hit%")
    else:
        print(l)
PY
