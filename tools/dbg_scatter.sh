#!/bin/bash
# scatter experiments: persistent grid sizes (TFIDF_SCATTER_WGS) and store/atomic ablations
set -o pipefail
mkdir -p gpurun_out
for cfg in "0 0" "0 256" "0 128" "0 64" "1 0" "2 0"; do
  set -- $cfg
  TFIDF_DEBUG_SCATTER=$1 TFIDF_SCATTER_WGS=$2 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 > gpurun_out/dbg.log 2>&1 || { tail -3 gpurun_out/dbg.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/dbg.log').read().strip().splitlines()[-1]); print('debug=$1 wgs=$2 scatter_ms', round(r['phases_ms']['ms_scatter'],3))"
done
