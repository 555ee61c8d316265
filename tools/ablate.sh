#!/bin/bash
# Tokenize-kernel ablation: time the kernel when each document stops after phase N.
set -o pipefail
for s in 1 2 3 4 5 0; do
  TFIDF_DEBUG_STOP=$s timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-queries --cpu-sample 0 > gpurun_out/ablate_$s.log 2>&1 || { echo "stop=$s failed"; tail -5 gpurun_out/ablate_$s.log; exit 1; }
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/ablate_$s.log').read().strip().splitlines()[-1]); print('stop=$s tokenize_ms=%.3f' % r['phases_ms']['ms_tokenize'])" 2>/dev/null || echo "stop=$s (commit error expected for partial runs)"; tail -1 gpurun_out/ablate_$s.log | cut -c1-200
done
