#!/bin/bash
# A/B of the side-stream dictionary mirror (TFIDF_MIRROR_MAIN=1: old placement)
# at cfg 2 and the book shape, after the parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_books.py tests/test_gpu_term_major.py tests/test_gpu_multirank.py > gpurun_out/abm_tests.log 2>&1 || { tail -30 gpurun_out/abm_tests.log; exit 1; }
tail -1 gpurun_out/abm_tests.log
for v in side main side main; do
  if [ $v = main ]; then export TFIDF_MIRROR_MAIN=1; else unset TFIDF_MIRROR_MAIN; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-queries --cpu-sample 0 --no-e2e > gpurun_out/abm_$v.log 2>&1 || { tail -5 gpurun_out/abm_$v.log; exit 2; }
  timeout -k 10 200 python -u bench.py --docs 300 --len-min 80000 --len-max 120000 --steps 5 --warmup 2 --no-queries --cpu-sample 0 --no-e2e > gpurun_out/abm_book_$v.log 2>&1 || { tail -5 gpurun_out/abm_book_$v.log; exit 3; }
  python3 -c "
import json
for f in ['gpurun_out/abm_$v.log','gpurun_out/abm_book_$v.log']:
    r=json.loads(open(f).read().strip().splitlines()[-1]); print('$v', f.split('/')[-1], 'ms/step %.3f' % r['ms_per_step'], 'phases total %.3f' % r['phases_ms']['ms_total'])"
done
