#!/bin/bash
# cfg-2 bench with queries (no CPU sample, no end-to-end): batch and single-query figures.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-e2e "$@" > gpurun_out/bq.json 2> gpurun_out/bq.err || { tail -5 gpurun_out/bq.err; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/bq.json').read().strip().splitlines()[-1]); q=r['queries']; print('batch runs', q['batch10k_device_ms_runs'], 'median', q['batch10k_device_ms'], 'single p50', q['single_top10_p50_ms'], 'all-hits 16t', q['threads16_all_hits_qps'])"
