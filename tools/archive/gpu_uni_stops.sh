#!/bin/bash
# Unicode wave path phase costs (cfg 2, every document non-ASCII): tokenize
# time with the kernel ending each document after phase 10 (stage), 11 (token
# list), 12 (table insert), 13 (dictionary), 0 (full).
set -o pipefail
mkdir -p gpurun_out
for s in 10 11 12 13 0; do
  TFIDF_DEBUG_STOP=$s timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 --no-e2e --unicode-frac ${FRAC:-1.0} > gpurun_out/ustop_$s.log 2> gpurun_out/ustop_$s.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/ustop_$s.err; exit $rc; }
  python3 -c "import json; r=json.loads(open('gpurun_out/ustop_$s.log').read().strip().splitlines()[-1]); print('stop $s tokenize %.2f ms' % r['phases_ms']['ms_tokenize'])"
done
