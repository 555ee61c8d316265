#!/bin/bash
# Kernel trace of the cfg-2 batch (bench with queries) under query-path knobs:
# SETS="name:VAR=val ..." (name only = defaults); prints each batch chunk's kernels.
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
for spec in ${SETS:-base}; do
  n=${spec%%:*}; e=""; [ "$n" != "$spec" ] && e=${spec#*:}
  env_args=${e//,/ }
  ( [ -n "$env_args" ] && export $env_args; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktb_$n -o kt -- python -u bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-e2e > gpurun_out/ktb_$n.log 2>&1 ) || { echo "$n failed"; tail -3 gpurun_out/ktb_$n.log; exit 1; }
  f=$(find gpurun_out/ktb_$n -name '*kernel_trace.csv' | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(x['Start_Timestamp']), int(x['End_Timestamp']), x['Kernel_Name']) for x in r)
idx = [i for i, e in enumerate(ev) if 'k_merge_topk_wave' in e[2]]
last = idx[-2:]
print('==', sys.argv[2])
for i in last:
    j = i
    while j > 0 and ('score_units' in ev[j - 1][2] or 'score_wunits' in ev[j - 1][2] or 'fillBuffer' in ev[j - 1][2]): j -= 1
    t0 = ev[j][0]
    for e in ev[j:i + 1]:
        print('  %8.3f %8.3f %s' % ((e[0] - t0) / 1e6, (e[1] - t0) / 1e6, e[2][:40]))
PY
done
