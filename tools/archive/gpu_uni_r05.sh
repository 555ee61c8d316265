#!/bin/bash
# Round 5: Unicode sparse path — parity (sparse + Unicode + identity + XCD units
# + books), then cfg 2 with 10 % / 100 % non-ASCII documents, sparse vs the
# whole-document scan (TFIDF_UW_FULL=1).  Every GPU step bounded.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_unicode_sparse.py tests/test_gpu_unicode.py tests/test_gpu_identity.py tests/test_gpu_xcd_units.py tests/test_gpu_books.py > gpurun_out/uni_tests.log 2>&1
rc=$?; tail -3 gpurun_out/uni_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/uni_tests.log | head -20; exit $rc; }
for f in 1.0 0.1; do
  for full in 0 1; do
    TFIDF_UW_FULL=$full timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-queries --cpu-sample 0 --no-e2e --unicode-frac $f > gpurun_out/uni_${f}_$full.log 2> gpurun_out/uni_${f}_$full.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/uni_${f}_$full.err; exit $rc; }
    python3 -c "import json; r=json.loads(open('gpurun_out/uni_${f}_$full.log').read().strip().splitlines()[-1]); print('frac $f full $full: ms/step %.2f tokenize %.2f unicode_docs %d' % (r['ms_per_step'], r['phases_ms']['ms_tokenize'], r['unicode_docs']))"
  done
done
