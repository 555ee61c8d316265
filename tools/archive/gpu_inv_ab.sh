#!/bin/bash
# Round 3: one-read inversion + fused single query — parity tests, then bench
# A/B against the round-2 inversion (build only), then one full bench (queries)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_units.py tests/test_gpu_operators.py} > gpurun_out/inv_tests.log 2>&1
rc=$?; tail -3 gpurun_out/inv_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/inv_tests.log | head -30; exit $rc; }
for v in new old; do
  if [ $v = old ]; then export TFIDF_INV_OLD=1; else unset TFIDF_INV_OLD; fi
  timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 --no-queries --no-e2e --cpu-sample 0 > gpurun_out/inv_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/inv_$v.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/inv_$v.log').read().strip().splitlines()[-1]); print('$v', round(r['ms_per_step'],3), {k: round(x, 3) for k, x in r['phases_ms'].items()})"
done
unset TFIDF_INV_OLD
timeout -k 10 300 python -u bench.py --no-e2e --cpu-sample 0 > gpurun_out/bench_q.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_q.log; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/bench_q.log').read().strip().splitlines()[-1]); print(round(r['ms_per_step'],3), {k: v for k, v in r['queries'].items() if k != 'roofline'})"
