#!/bin/bash
# Round 5: book units with non-ASCII words by the wave rules
# (k_tokenize_chunk<UNI>) — parity, then 300 books with one é word per
# 2 KB with the wave rules on / off (TFIDF_NO_UNIWAVE=1) and the ASCII books.
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_uni_wave.py tests/test_gpu_books.py tests/test_gpu_unicode.py tests/test_gpu_identity.py > gpurun_out/unib_tests.log 2>&1
rc=$?; tail -2 gpurun_out/unib_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/unib_tests.log | head -20; exit $rc; }
B="--steps 10 --warmup 2 --docs 300 --len-min 80000 --len-max 120000 --no-queries --no-e2e --cpu-sample 0"
for v in uni uwoff ascii; do
  A="$B --unicode-every 2048"; [ $v = ascii ] && A="$B"
  if [ $v = uwoff ]; then export TFIDF_NO_UNIWAVE=1; else unset TFIDF_NO_UNIWAVE; fi
  timeout -k 10 300 python -u bench.py $A > gpurun_out/unib_$v.log 2> gpurun_out/unib_$v.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/unib_$v.err; exit $rc; }
  python3 -c "import json; r=json.loads(open('gpurun_out/unib_$v.log').read().strip().splitlines()[-1]); print('books $v: ms/step %.3f long %.3f' % (r['ms_per_step'], r['phases_ms']['ms_long']))"
done
