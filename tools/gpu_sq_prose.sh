#!/bin/bash
# SQ counters of the tokenizer kernels: cfg-2 prose (UNI-first after the first
# commit) against plain ASCII.  One counter set per pass.
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/sq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pr in 1 0; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_tokenize" -d $O/a_$pr -o a --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-queries --no-e2e --cpu-sample 0 --prose $pr > $O/a_$pr.log 2>&1 || { echo "a $pr failed"; tail -3 $O/a_$pr.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --kernel-include-regex "k_tokenize" -d $O/b_$pr -o b --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-queries --no-e2e --cpu-sample 0 --prose $pr > $O/b_$pr.log 2>&1 || { echo "b $pr failed"; tail -3 $O/b_$pr.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for pr in (1, 0):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for s in ("a", "b"):
        for f in glob.glob("/root/repo/gpurun_out/sq/%s_%d/**/*counter_collection.csv" % (s, pr), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"][:46]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        if d.get("SQ_WAVE_CYCLES", 0) < 1e6: continue
        print("prose", pr, k)
        print("   " + "  ".join("%s=%.3g" % (c, v) for c, v in sorted(d.items())))
PY
