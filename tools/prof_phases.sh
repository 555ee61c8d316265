#!/bin/bash
# PMC counters of the wave tokenize kernel per phase: runs with
# TFIDF_DEBUG_STOP in STOPS (default "2 3 4 0") and prints per-doc deltas
# between consecutive stops.  DOCS docs (default 200k).  KRE: kernel name
# regex (default tokenize_wave; "tokenize_wave<false, false, true>" for the
# UNI pass alone), BARGS: extra bench.py arguments (e.g. --unicode-frac 1.0).
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/prof_phases; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
STOPS=${STOPS:-"2 3 4 0"}; DOCS=${DOCS:-200000}; KRE=${KRE:-tokenize_wave}; BARGS=${BARGS:-}
[ -f $O/counters.txt ] || timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_BUSY_CYCLES"
for s in $STOPS; do
 for g in 1 2; do
  if [ $g = 1 ]; then C=$G1; else C=$G2; fi
  TFIDF_DEBUG_STOP=$s timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -d $O/s${s}g$g -o p --output-format csv -- python3 $R/bench.py --docs $DOCS --steps 1 --warmup 0 --no-queries --cpu-sample 0 $BARGS > $O/s${s}g$g.log 2>&1 || { echo "pmc s=$s g=$g failed"; tail -3 $O/s${s}g$g.log; exit 2; }
 done
done
python3 - $O $DOCS $STOPS <<'PY'
import csv, collections, glob, sys
O, N = sys.argv[1], int(sys.argv[2]); stops = sys.argv[3:]
def agg(s):
    # per launch: bench.py runs the build more than once (timed step + the
    # end-to-end leg), so each counter is averaged over the dispatches
    d = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for f in glob.glob("%s/s%sg*/*counter_collection.csv" % (O, s)):
        for r in csv.DictReader(open(f)):
            d[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]].add(r["Dispatch_Id"])
    return {k: v / max(len(n[k]), 1) for k, v in d.items()}
A = [agg(s) for s in stops]
keys = sorted(set().union(*[set(a) for a in A]))
print("%-24s" % "per doc" + "".join("%14s" % ("stop%s" % s) for s in stops) + "   deltas")
for k in keys:
    vals = [a.get(k, 0) / N for a in A]
    print("%-24s" % k + "".join("%14.1f" % v for v in vals) + "   " + " ".join("%.1f" % (vals[i] - vals[i - 1]) for i in range(1, len(vals))))
PY
