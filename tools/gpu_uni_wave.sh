#!/bin/bash
# Round 5: non-ASCII documents by the wave rules (k_tokenize_wave<UNI>) —
# parity (new + the existing Unicode suites), then cfg 2 with 10 % / 100 %
# non-ASCII documents with the wave rules on and off (TFIDF_NO_UNIWAVE=1),
# and the all-ASCII cfg-2 step.  Every GPU step bounded.
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_uni_wave.py tests/test_gpu_unicode_sparse.py tests/test_gpu_unicode.py tests/test_gpu_identity.py tests/test_gpu_xcd_units.py tests/test_gpu_books.py tests/test_gpu_pack.py > gpurun_out/uniw_tests.log 2>&1
rc=$?; tail -3 gpurun_out/uniw_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/uniw_tests.log | head -30; exit $rc; }
for f in 1.0 0.1 0.0; do
  for off in 0 1; do
    [ "$f" = "0.0" ] && [ $off = 1 ] && continue
    if [ $off = 1 ]; then export TFIDF_NO_UNIWAVE=1; else unset TFIDF_NO_UNIWAVE; fi
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-queries --cpu-sample 0 --no-e2e --unicode-frac $f > gpurun_out/uniw_${f}_$off.log 2> gpurun_out/uniw_${f}_$off.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/uniw_${f}_$off.err; exit $rc; }
    python3 -c "import json; r=json.loads(open('gpurun_out/uniw_${f}_$off.log').read().strip().splitlines()[-1]); print('frac $f no_uniwave $off: ms/step %.2f tokenize %.2f unicode_docs %d' % (r['ms_per_step'], r['phases_ms']['ms_tokenize'], r['unicode_docs']))"
  done
done
