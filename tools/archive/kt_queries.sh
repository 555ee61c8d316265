#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ktq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_score|k_merge|k_hits" -d $O -o kt --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-sample 0 --no-e2e > $O/kt.log 2>&1 || { echo kt failed; tail -3 $O/kt.log; exit 1; }
python3 - $O <<'P'
import csv,sys,glob
for f in glob.glob(sys.argv[1]+'/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)): print("%-50s %6s %9.2f us" % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))
P
