#!/bin/bash
# Round 5: phase stops (TFIDF_DEBUG_STOP 1..4, 0) at cfg 2 with all documents
# non-ASCII (one simple é word each: k_tokenize_wave<UNI>) and all ASCII.
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
mkdir -p gpurun_out
for f in 1.0 0.0; do
  for st in 1 2 3 4 0; do
    TFIDF_DEBUG_STOP=$st timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 --no-e2e --unicode-frac $f > gpurun_out/uwst_${f}_$st.log 2> gpurun_out/uwst_${f}_$st.err
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/uwst_${f}_$st.err; exit $rc; }
    python3 -c "import json; r=json.loads(open('gpurun_out/uwst_${f}_$st.log').read().strip().splitlines()[-1]); print('frac $f stop $st tokenize %.2f' % r['phases_ms']['ms_tokenize'])"
  done
done
