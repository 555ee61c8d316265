#!/bin/bash
# Tokenizer phase probe by wall time: cfg-2 bench with TFIDF_DEBUG_STOP = each of
# STOPS (3 histogram, 4 dictionary, 5 everything but the row / per-document
# stores, 0 full); ms_tokenize per stop.  Timing only: rows are incomplete.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rnd in 1 2; do
for st in ${STOPS:-0 3 4 5}; do
  if [ $st = 0 ]; then unset TFIDF_DEBUG_STOP; else export TFIDF_DEBUG_STOP=$st; fi
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-queries --no-e2e --cpu-sample 0 $ARGS > gpurun_out/stop.log 2>&1 || { echo "stop $st failed"; tail -5 gpurun_out/stop.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/stop.log').read().strip().splitlines()[-1]); print('stop $st', round(r['phases_ms']['ms_tokenize'], 3))"
done
done
