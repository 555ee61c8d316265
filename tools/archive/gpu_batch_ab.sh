#!/bin/bash
# batch pipeline: tests, then host split per chunk count
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_units.py tests/test_gpu_operators.py tests/test_gpu_fullsize.py > gpurun_out/b_tests.log 2>&1
rc=$?; tail -2 gpurun_out/b_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/b_tests.log | head -30; exit $rc; }
for c in 1 2 4 8; do
  TFIDF_BATCH_CHUNKS=$c TFIDF_HOST_TIMING=1 timeout -k 10 300 python3 tools/time_batch_host.py > gpurun_out/b_$c.log 2>&1 || { echo "chunks $c failed"; tail -3 gpurun_out/b_$c.log; exit 1; }
  echo "chunks $c"; grep -E "^batch 10000|qps" gpurun_out/b_$c.log | tail -4
done
