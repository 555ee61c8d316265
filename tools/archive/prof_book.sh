#!/bin/bash
# cfg-1 shape (300 book-sized documents): kernel-trace summary of the bench's builds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/prof_book; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --docs 300 --len-min 80000 --len-max 120000 --steps 5 --warmup 2 --no-queries --cpu-sample 0 --no-e2e > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("%-44s calls=%4s avg_ms=%8.4f total_ms=%8.3f" % (r["Name"].split("(")[0][-44:], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
grep -h '"metric"' $O/kt.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['ms_per_step'], r['phases_ms'])"
