#!/bin/bash
# Tokenize-kernel ablation: kernel time when each document stops after phase N
# (TFIDF_DEBUG_STOP: 1 staged, 2 classified + spans, 3 histogram, 4 dictionary
# lookups, 0 full).  Reduced corpus size via DOCS (default 1M).
set -o pipefail
mkdir -p gpurun_out
for s in ${STOPS:-1 2 3 4 0}; do
  TFIDF_DEBUG_STOP=$s timeout -k 10 200 python -u bench.py --docs ${DOCS:-1000000} --steps 2 --warmup 1 --no-queries --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/ablate_$s.log 2>&1
  python3 -c "import json; r=json.loads(open('gpurun_out/ablate_$s.log').read().strip().splitlines()[-1]); print('stop=$s tokenize_ms=%.3f' % r['phases_ms']['ms_tokenize'])" 2>/dev/null || { echo "stop=$s: no result"; tail -3 gpurun_out/ablate_$s.log; }
done
