#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of the build-only bench for
# library variants: VARIANTS="name[:bench args] ..." where name = base (the
# tree's lib) or a lib_var/<name>/libtfidf.so; per-kernel averages printed.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out lib_var/base
cp tf-idf-distributed-system_amd/lib/libtfidf.so lib_var/base/libtfidf.so
export TMPDIR=/tmp
rc=0
for spec in $VARIANTS; do
  v=${spec%%:*}; a=""; [ "$v" != "$spec" ] && a=${spec#*:}
  cp lib_var/$v/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
  echo "== $v $a"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$v -o kt -- python -u bench.py --steps 5 --warmup 1 --no-queries --no-e2e --cpu-sample 0 ${a//,/ } > gpurun_out/kt_$v.log 2>&1 || { rc=$?; echo "$v failed"; tail -5 gpurun_out/kt_$v.log; break; }
  f=$(find gpurun_out/kt_$v -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in r[:14]: print('%-40s %6s calls  avg %8.3f ms' % (x['Name'][:40], x['Calls'], float(x['AverageNs'])/1e6))"
done
cp lib_var/base/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
exit $rc
