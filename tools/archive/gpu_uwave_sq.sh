#!/bin/bash
# SQ counters of k_tokenize_uwave on cfg 2 with every document non-ASCII (one PMC pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY --kernel-include-regex "k_tokenize_uwave" -d $R/gpurun_out/sq_uwave -o sq --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --docs 200000 --no-queries --no-e2e --cpu-sample 0 --unicode-frac 1.0 > $R/gpurun_out/sq_uwave.log 2>&1 || { echo "sq failed"; tail -3 $R/gpurun_out/sq_uwave.log; exit 1; }
f=$(find $R/gpurun_out/sq_uwave -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    tot[r["Counter_Name"]] += float(r["Counter_Value"])
docs = 200000
for k in sorted(tot):
    print("%-20s total %.4g  per doc %.1f" % (k, tot[k], tot[k] / docs))
PY
