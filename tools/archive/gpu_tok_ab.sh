#!/bin/bash
# Tokenizer A/B: in-tree build vs tools/archive/variants/*.so, cfg 2 and cfg-5 shape
# builds alternated (ROUNDS), after the wave-path parity tests (TESTS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
if [ "${TESTS:-x}" != none ]; then
  timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_pack.py tests/test_gpu_identity.py tests/test_gpu_unicode.py} > gpurun_out/tok_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/tok_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/tok_tests.log | head -30; exit $rc; }
fi
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
for rnd in $(seq 1 ${ROUNDS:-2}); do
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  for shape in ${BASESHAPE-cfg2} ${SHAPES:-cfg5}; do
    A="--steps 5 --warmup 2"
    [ $shape = cfg5 ] && A="--steps 3 --warmup 1 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000"
    [ $shape = book ] && A="--steps 5 --warmup 2 --docs 300 --len-min 80000 --len-max 120000"
    timeout -k 10 300 python -u bench.py $A --no-queries --no-e2e --cpu-sample 0 > gpurun_out/tok.log 2>&1 || { echo "$v $shape failed"; tail -3 gpurun_out/tok.log; cp /tmp/libtfidf_base.so $L; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/tok.log').read().strip().splitlines()[-1]); print('%-28s %s' % ('$v', '$shape'), round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x})"
  done
done
done
cp /tmp/libtfidf_base.so $L
