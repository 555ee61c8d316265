#!/bin/bash
# Tokenizer occupancy probe: persistent-grid workgroups per CU (1 wave each)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for w in ${WPC:-8 4 6 8}; do
  TFIDF_WAVE_WGS_PER_CU=$w timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-queries --no-e2e --cpu-sample 0 > gpurun_out/occ.log 2>&1 || { echo "wpc $w failed"; tail -3 gpurun_out/occ.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/occ.log').read().strip().splitlines()[-1]); print('wgs/CU $w', round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x})"
done
