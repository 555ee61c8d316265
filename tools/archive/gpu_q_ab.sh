#!/bin/bash
# query A/B: in-tree build vs tools/archive/variants/*.so (single top-10, all hits, 10 k batch)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
if [ "${TESTS:-x}" != none ]; then
  timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_units.py tests/test_gpu_fused.py tests/test_gpu_operators.py tests/test_gpu_parity.py} > gpurun_out/q_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/q_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/q_tests.log | head -30; exit $rc; }
fi
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
for rnd in $(seq 1 ${ROUNDS:-2}); do
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-e2e --cpu-sample 0 ${ARGS:-} > gpurun_out/q.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/q.log; cp /tmp/libtfidf_base.so $L; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/q.log').read().strip().splitlines()[-1]); q=r['queries']; print('%-26s' % '$v', {k: round(q[k],4) for k in ('single_top10_qps','single_top10_p50_ms','single_top10_device_ms_avg','single_all_hits_device_ms_avg','batch10k_top10_qps','batch10k_device_ms')})"
done
done
cp /tmp/libtfidf_base.so $L
