#!/bin/bash
# Tokenizer arena A/B: parity on the in-tree build, then cfg-2 / cfg-5 builds for
# the in-tree build at 10 and 8 workgroups per CU and the variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
L=tf-idf-distributed-system_amd/lib/libtfidf.so
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_pack.py tests/test_gpu_identity.py tests/test_gpu_unicode.py tests/test_gpu_books.py} > gpurun_out/w10_tests.log 2>&1
rc=$?; tail -1 gpurun_out/w10_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/w10_tests.log | head -20; exit $rc; }
cp $L /tmp/base.so
for rnd in 1 2; do
for cfg in "base 10" "base 8" "tools/archive/variants/w2.so 8" "tools/archive/variants/head.so 8"; do
  set -- $cfg
  if [ $1 = base ]; then cp /tmp/base.so $L; else cp $1 $L; fi
  for shape in cfg2 cfg5; do
    A="--steps 5 --warmup 2"
    [ $shape = cfg5 ] && A="--steps 3 --warmup 1 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000"
    TFIDF_WAVE_WGS_PER_CU=$2 timeout -k 10 300 python -u bench.py $A --no-queries --no-e2e --cpu-sample 0 > gpurun_out/w10.log 2>&1 || { echo "$1 $2 $shape failed"; tail -3 gpurun_out/w10.log; cp /tmp/base.so $L; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/w10.log').read().strip().splitlines()[-1]); print('%-26s %3s %s' % ('$1', '$2', '$shape'), round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x > 0.01})"
  done
done
done
cp /tmp/base.so $L
