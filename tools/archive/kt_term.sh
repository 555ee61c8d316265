#!/bin/bash
# kernel-trace summaries of the cfg-5 shape build, onesweep and old LSD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd /tmp && export TMPDIR=/tmp
for v in new old; do
  O=$R/gpurun_out/kt_term_$v; mkdir -p $O
  if [ $v = old ]; then export TFIDF_TERM_LSD_OLD=1; else unset TFIDF_TERM_LSD_OLD; fi
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-queries --no-e2e --cpu-sample 0 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000 > $O/log 2>&1 || { echo "kt $v failed"; tail -5 $O/log; exit 1; }
  python3 - $O $v <<'P'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1]+'/kt_kernel_stats.csv')))
for r in rows[:14]: print("%-4s %-56s %5s %10.1f us" % (sys.argv[2], r['Name'][:56], r['Calls'], float(r['AverageNs'])/1e3))
P
done
