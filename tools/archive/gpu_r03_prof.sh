#!/bin/bash
# Round-3 profile refresh: prof_round (kernel trace of the default bench, PMC
# traffic, SQ counters), then kernel traces of the cfg-5 and book shapes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=r03 SQ=1 timeout -k 10 900 bash tools/prof_round.sh > gpurun_out/prof_r03.log 2>&1 || { echo "prof_round failed"; tail -20 gpurun_out/prof_r03.log; exit 1; }
tail -30 gpurun_out/prof_r03.log
cd /tmp && export TMPDIR=/tmp
for shape in cfg5 book; do
  A="--steps 3 --warmup 1 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000"
  [ $shape = book ] && A="--steps 5 --warmup 2 --docs 300 --len-min 80000 --len-max 120000"
  O=$R/gpurun_out/kt_$shape; mkdir -p $O
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py $A --no-queries --no-e2e --cpu-sample 0 > $O/bench.log 2>&1 || { echo "kt $shape failed"; tail -5 $O/bench.log; exit 1; }
  echo "kt $shape ok"
done
