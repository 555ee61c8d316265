#!/bin/bash
# single-query A/B: host merge (one launch), split (merge kernel), wg (last-workgroup merge), round-2 path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_fused.py} > gpurun_out/q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/q_tests.log | head -30; exit $rc; }
for v in host split wg old; do
  unset TFIDF_FUSED_MODE TFIDF_NO_FUSED
  [ $v = split ] && export TFIDF_FUSED_MODE=split
  [ $v = wg ] && export TFIDF_FUSED_MODE=wg
  [ $v = old ] && export TFIDF_NO_FUSED=1
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-e2e --cpu-sample 0 --batch-queries 1000 > gpurun_out/q_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/q_$v.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/q_$v.log').read().strip().splitlines()[-1]); q=r['queries']; print('$v', round(r['ms_per_step'],3), {k: round(q[k],4) for k in ('single_top10_qps','single_top10_p50_ms','single_top10_p99_ms','single_top10_device_ms_avg')})"
done
