#!/bin/bash
# All-hits ordering A/B: parity tests, then the bench's query section with the
# 8-run group merge (default) and with the pairwise levels only (TFIDF_HITS_PAIRWISE=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
if [ "${TESTS:-x}" != none ]; then
  timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_hits_merge.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_operators.py} > gpurun_out/hits_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/hits_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/hits_tests.log | head -30; exit $rc; }
fi
for rnd in 1 2; do
for mode in group pairwise; do
  E=""; [ $mode = pairwise ] && E="TFIDF_HITS_PAIRWISE=1"
  env $E timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-e2e > gpurun_out/hits_bench.log 2>&1 || { echo "$mode failed"; tail -3 gpurun_out/hits_bench.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/hits_bench.log').read().strip().splitlines()[-1]); q=r['queries']; print('$mode', {k: round(q[k], 4) for k in q if 'all_hits' in k})"
done
done
