#!/bin/bash
# cfg-5 shape: documents per packed tokenizer window (TFIDF_PACK_DOCS) vs tokenize time.
set -o pipefail
mkdir -p gpurun_out
for p in ${PACKS:-5 6 7 8}; do
  TFIDF_PACK_DOCS=$p timeout -k 10 200 python -u bench.py --docs 6250000 --vocab 5000000 --len-min 48 --len-max 80 --steps 2 --warmup 1 --no-queries --cpu-sample 0 --no-e2e > gpurun_out/pack_$p.log 2>&1 || { echo "pack=$p failed"; tail -3 gpurun_out/pack_$p.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/pack_$p.log').read().strip().splitlines()[-1]); print('pack=$p tokenize_ms=%.3f step_ms=%.2f retried=%s per_window=%s' % (r['phases_ms']['ms_tokenize'], r['ms_per_step'], r['pack_retried_docs'], r['tokenizer_docs_per_window']))"
done
