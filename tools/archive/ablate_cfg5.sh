#!/bin/bash
# Tokenizer phase ablation at the cfg-5 shape (TFIDF_DEBUG_STOP; see tools/prof_round.sh)
set -o pipefail
mkdir -p gpurun_out
for s in 1 2 3 4 0; do
  TFIDF_DEBUG_STOP=$s timeout -k 10 200 python -u bench.py --docs 6250000 --vocab 5000000 --len-min 48 --len-max 80 \
    --steps 2 --warmup 1 --no-queries --cpu-sample 0 --no-e2e > gpurun_out/ablate5_$s.log 2>&1 || { echo "stop=$s failed"; tail -3 gpurun_out/ablate5_$s.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/ablate5_$s.log').read().strip().splitlines()[-1]); print('stop=$s tokenize_ms=%.3f' % r['phases_ms']['ms_tokenize'])"
done
