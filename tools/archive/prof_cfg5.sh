#!/bin/bash
# cfg-5 shape: kernel-trace summary of one build + tokenizer phase ablation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/prof_cfg5; mkdir -p $O
ARGS="--docs 6250000 --vocab 5000000 --len-min 48 --len-max 80 --no-queries --cpu-sample 0 --no-e2e"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 $ARGS > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-44s calls=%4s avg_ms=%8.4f total_ms=%8.3f" % (r["Name"].split("(")[0][-44:], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
cd $R
for s in 1 2 3 4 0; do
  TFIDF_DEBUG_STOP=$s timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 $ARGS > $O/ablate_$s.log 2>&1 || { echo "stop=$s failed"; tail -3 $O/ablate_$s.log; exit 1; }
  python3 -c "import json; r=json.loads(open('$O/ablate_$s.log').read().strip().splitlines()[-1]); print('stop=$s tokenize_ms=%.3f' % r['phases_ms']['ms_tokenize'])"
done
