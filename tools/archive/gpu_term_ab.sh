#!/bin/bash
# term-major (cfg 5 / books) inversion: parity tests, then cfg-5 shape + books bench, onesweep vs old LSD
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
if [ "${TESTS:-x}" != none ]; then
  timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_term_major.py tests/test_gpu_books.py tests/test_gpu_fullsize.py} > gpurun_out/term_tests.log 2>&1
  rc=$?; tail -2 gpurun_out/term_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/term_tests.log | head -30; exit $rc; }
fi
for rnd in 1 2; do
for v in new old; do
  if [ $v = old ]; then export TFIDF_TERM_LSD_OLD=1; else unset TFIDF_TERM_LSD_OLD; fi
  for shape in cfg5 books; do
    A="--steps 3 --warmup 1 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000"
    [ $shape = books ] && A="--steps 5 --warmup 2 --docs 300 --len-min 80000 --len-max 120000"
    timeout -k 10 300 python -u bench.py $A --no-queries --no-e2e --cpu-sample 0 > gpurun_out/term.log 2>&1 || { echo "$v $shape failed"; tail -3 gpurun_out/term.log; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/term.log').read().strip().splitlines()[-1]); print('%-5s %-6s' % ('$v', '$shape'), round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x})"
  done
done
done
