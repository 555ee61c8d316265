#!/bin/bash
# 300 books, ASCII and prose: bench lines + kernel traces (round 6).
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
B="python -u bench.py --steps 10 --warmup 2 --no-queries --no-e2e --cpu-sample 0 --docs 300 --len-min 80000 --len-max 120000"
for pr in 0 1; do
  timeout -k 10 300 $B --prose $pr > gpurun_out/books_$pr.json 2> gpurun_out/books_$pr.err || { tail -3 gpurun_out/books_$pr.err; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/books_$pr.json').read().strip().splitlines()[-1]); print('books prose $pr step %.3f long %.3f chunked %s/%s' % (r['ms_per_step'], r['phases_ms']['ms_long'], r['long_chunked'], r['long_docs']))"
done
VARIANTS="base:--docs,300,--len-min,80000,--len-max,120000,--prose,1" bash tools/kt_ab.sh
