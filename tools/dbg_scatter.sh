#!/bin/bash
# scatter ablations: TFIDF_DEBUG_SCATTER 0 (normal) / 2 (atomics, no stores)
set -o pipefail
mkdir -p gpurun_out
for v in 0 2; do
  TFIDF_DEBUG_SCATTER=$v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 > gpurun_out/dbg.log 2>&1 || { tail -3 gpurun_out/dbg.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/dbg.log').read().strip().splitlines()[-1]); print('debug=$v', {k: round(x,3) for k,x in r['phases_ms'].items()})"
done
