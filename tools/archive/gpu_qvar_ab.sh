#!/bin/bash
# Query A/B: parity (TESTS) per library, then the cfg-2 bench with its query
# section (batch device time, single-query latency) for the in-tree build and
# each tools/archive/variants/*.so, ROUNDS times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread $TESTS > gpurun_out/qvar_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/qvar_tests.log)"; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/qvar_tests.log | head -20; cp /tmp/libtfidf_base.so $L; exit $rc; }
done
for rnd in $(seq 1 ${ROUNDS:-2}); do
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-e2e --cpu-sample 0 > gpurun_out/qvar.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/qvar.log; cp /tmp/libtfidf_base.so $L; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/qvar.log').read().strip().splitlines()[-1]); q=r['queries']; print('%-28s' % '$v', {k: round(q[k], 4) for k in ('batch10k_device_ms', 'batch10k_top10_qps', 'single_top10_p50_ms', 'single_all_hits_device_ms_avg')})"
done
done
cp /tmp/libtfidf_base.so $L
