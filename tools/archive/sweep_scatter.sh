#!/bin/bash
# cfg-2 block-major scatter knobs (A/B environment variables), two rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rnd in 1 2; do
for E in "X=0" "TFIDF_SORT_SPW=2" "TFIDF_SORT_SPW=8" "TFIDF_SORT_THREADS=256" "TFIDF_SORT_THREADS=1024" "TFIDF_PART_THREADS=512"; do
  env $E timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-queries --no-e2e --cpu-sample 0 > gpurun_out/sweep.log 2>&1 || { echo "$E failed"; tail -3 gpurun_out/sweep.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]); print('%-26s' % '$E', round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if k in ('ms_df','ms_scatter')})"
done
done
