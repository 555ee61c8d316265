#!/bin/bash
# Batch-scoring A/B over library variants: for the in-tree build and each
# tools/archive/variants/*.so, the unit / operator parity tests, then the 10 k-query
# batch timing (tools/time_batch_host.py: device ms per batch), ROUNDS times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_units.py tests/test_gpu_operators.py ${TESTS:-} > gpurun_out/bv_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/bv_tests.log)"; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/bv_tests.log | head -20; cp /tmp/libtfidf_base.so $L; exit $rc; }
done
for rnd in $(seq 1 ${ROUNDS:-2}); do
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  timeout -k 10 300 python3 tools/time_batch_host.py > gpurun_out/bv.log 2>&1 || { echo "$v batch failed"; tail -3 gpurun_out/bv.log; cp /tmp/libtfidf_base.so $L; exit 1; }
  echo "$v: $(grep -E 'device' gpurun_out/bv.log | tail -2 | tr '\n' ' ')"
done
done
cp /tmp/libtfidf_base.so $L
