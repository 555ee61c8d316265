#!/bin/bash
# Tokenizer phase times at cfg 2 (TFIDF_DEBUG_STOP 1 2 3 4 0: cumulative).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for s in 1 2 3 4 0; do
  TFIDF_DEBUG_STOP=$s timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 --no-e2e > gpurun_out/ablate_$s.log 2>&1 || { echo "stop=$s failed"; tail -3 gpurun_out/ablate_$s.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/ablate_$s.log').read().strip().splitlines()[-1]); print('stop=$s tokenize_ms=%.3f' % r['phases_ms']['ms_tokenize'])"
done
