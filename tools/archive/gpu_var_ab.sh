#!/bin/bash
# Variant A/B with parity per variant: for the in-tree build and each
# tools/archive/variants/*.so, run TESTS (bounded) then the bench SHAPES, ROUNDS times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread $TESTS > gpurun_out/var_tests.log 2>&1
  rc=$?; echo "$v tests: $(tail -1 gpurun_out/var_tests.log)"; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/var_tests.log | head -20; cp /tmp/libtfidf_base.so $L; exit $rc; }
done
for rnd in $(seq 1 ${ROUNDS:-2}); do
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  for shape in ${SHAPES:-cfg2}; do
    A="--steps 5 --warmup 2"
    [ $shape = cfg5 ] && A="--steps 3 --warmup 1 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000"
    [ $shape = book ] && A="--steps 5 --warmup 2 --docs 300 --len-min 80000 --len-max 120000"
    [ $shape = bookuni ] && A="--steps 5 --warmup 2 --docs 300 --len-min 80000 --len-max 120000 --unicode-every 2048"
    [ $shape = uni10 ] && A="--steps 5 --warmup 2 --unicode-frac 0.1"
    [ $shape = uni100 ] && A="--steps 3 --warmup 1 --unicode-frac 1.0"
    timeout -k 10 300 python -u bench.py $A --no-queries --no-e2e --cpu-sample 0 > gpurun_out/tok.log 2>&1 || { echo "$v $shape failed"; tail -3 gpurun_out/tok.log; cp /tmp/libtfidf_base.so $L; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/tok.log').read().strip().splitlines()[-1]); print('%-28s %s' % ('$v', '$shape'), round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x > 0.01})"
  done
done
done
cp /tmp/libtfidf_base.so $L
