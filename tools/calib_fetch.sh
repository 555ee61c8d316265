#!/bin/bash
# FETCH_SIZE calibration for random 16 / 32 / 128 B probes (tools/calib_fetch.hip):
# one rocprofv3 pass per counter group, per-dispatch values against the
# requested bytes.  Output: gpurun_out/calib_fetch/summary.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/calib_fetch; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B=$R/tools/bin/calib_fetch
timeout -k 10 120 $B > $O/order.txt 2>&1 || { echo "plain run failed"; cat $O/order.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- $B > $O/kt.log 2>&1 || { echo "kt failed"; tail -3 $O/kt.log; exit 1; }
i=0
for C in "FETCH_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B" "TCC_EA0_RDREQ_DRAM TCC_EA0_RDREQ_DRAM_32B" "TCC_HIT TCC_MISS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $O/p$i -o p --output-format csv -- $B > $O/p$i.log 2>&1 || { echo "pmc $C failed"; tail -3 $O/p$i.log; exit 1; }
done
python3 - $O <<'PY' | tee $O/summary.txt
import csv, glob, sys, collections
O = sys.argv[1]
order = [l.split() for l in open(O + "/order.txt") if l.strip() and not l.startswith("dispatch")]
vals = collections.defaultdict(dict)        # dispatch index -> counter -> value
for f in sorted(glob.glob(O + "/p*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "k_" in r["Kernel_Name"]]   # (not the memset's fill kernel)
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})
    rank = {d: k for k, d in enumerate(ids)}
    for r in rows:
        vals[rank[int(r["Dispatch_Id"])]][r["Counter_Name"]] = vals[rank[int(r["Dispatch_Id"])]].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
dur = []
for f in glob.glob(O + "/kt/**/*kernel_trace.csv", recursive=True):
    rows = sorted([r for r in csv.DictReader(open(f)) if "k_" in r["Kernel_Name"]], key=lambda r: int(r["Dispatch_Id"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print("%-22s %12s %8s %10s %10s %10s %10s %10s %10s %9s" % ("launch", "bytes req", "ms", "FETCH/req", "RDREQ", "RDREQ32", "RDREQ64", "DRAM", "DRAM32", "L2 hit%"))
for k, (name, probes, req) in enumerate(order):
    v = vals.get(k, {}); req = float(req)
    fetch = v.get("FETCH_SIZE", 0) * 1024.0
    hit, miss = v.get("TCC_HIT", 0), v.get("TCC_MISS", 0)
    print("%-22s %12.4g %8.3f %10.3f %10.4g %10.4g %10.4g %10.4g %10.4g %9.1f" % (
        name, req, dur[k] if k < len(dur) else 0, fetch / req, v.get("TCC_EA0_RDREQ", 0), v.get("TCC_EA0_RDREQ_32B", 0),
        v.get("TCC_EA0_RDREQ_64B", 0), v.get("TCC_EA0_RDREQ_DRAM", 0), v.get("TCC_EA0_RDREQ_DRAM_32B", 0),
        100.0 * hit / max(hit + miss, 1)))
PY
