#!/bin/bash
# Round 6: phase stops (TFIDF_DEBUG_STOP) at cfg 2, prose (--prose 1: every
# document takes k_tokenize_wave<UNI>; stop 5 = after the prose window check,
# 6 = after the classifier) and plain ASCII.
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
mkdir -p gpurun_out
run() {
  TFIDF_DEBUG_STOP=$2 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 --no-e2e --prose $1 > gpurun_out/prst_$1_$2.log 2> gpurun_out/prst_$1_$2.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/prst_$1_$2.err; return $rc; }
  python3 -c "import json; r=json.loads(open('gpurun_out/prst_$1_$2.log').read().strip().splitlines()[-1]); print('prose $1 stop $2 tokenize %.2f' % r['phases_ms']['ms_tokenize'])"
}
for st in 5 6 2 3 4 0; do run 1 $st || exit $?; done
TFIDF_NO_UNIFIRST=1 run 1 0 || exit $?
for st in 1 2 0; do run 0 $st || exit $?; done
