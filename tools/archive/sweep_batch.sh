#!/bin/bash
# 10 k-query batch knobs (A/B environment variables) on the cfg-2 index, two rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rnd in 1 2; do
for E in ${ENVS:-"X=0" "TFIDF_BATCH_CHUNKS=1" "TFIDF_WUNIT_LIGHT=200" "TFIDF_WUNIT_LIGHT=800" "TFIDF_UNIT_WG_PER_CU=1" "TFIDF_UNIT_WG_PER_CU=3"}; do
  env $E timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-e2e > gpurun_out/sweepb.log 2>&1 || { echo "$E failed"; tail -3 gpurun_out/sweepb.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/sweepb.log').read().strip().splitlines()[-1]); q=r['queries']; print('%-26s' % '$E', {k: round(q[k], 3) for k in ('batch10k_top10_qps','batch10k_device_ms','batch10k_scoring_ms')})"
done
done
