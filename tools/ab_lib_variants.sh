#!/bin/bash
# A/B of library builds (lib_var/<name>/libtfidf.so, built beside lib/ with
# different compile-time constants) on one command: each variant's .so is
# copied over lib/libtfidf.so for its run (a fresh process loads it), the
# default build is restored at the end.  CMD: the measurement (default: the
# 10 k-query batch timer).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out lib_var/base
CMD=${CMD:-"python -u tools/time_batch_host.py"}
cp tf-idf-distributed-system_amd/lib/libtfidf.so lib_var/base/libtfidf.so
rc=0
for round in 1 2; do
  for v in base $VARIANTS; do
    cp lib_var/$v/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
    echo "== $v (round $round)"
    timeout -k 10 240 $CMD > gpurun_out/abv_$v.log 2>&1 || { rc=$?; echo "$v failed"; tail -5 gpurun_out/abv_$v.log; break 2; }
    tail -3 gpurun_out/abv_$v.log
  done
done
cp lib_var/base/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
exit $rc
