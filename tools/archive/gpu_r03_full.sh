#!/bin/bash
# Round 3: whole GPU suite (incl. the full-size 8-shard tests), smoke, default
# bench, kernel-trace summary of the bench.  Every GPU step bounded.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread -s ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
tail -1 gpurun_out/bench.log | cut -c1-900
[ -n "${NO_KT:-}" ] && exit 0
O=$R/gpurun_out/kt_r03; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py > $O/kt_bench.log 2>&1 || { echo "kt failed"; tail -5 $O/kt_bench.log; exit 1; }
echo kt ok
