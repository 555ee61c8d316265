#!/bin/bash
# cfg-2 build (no queries) per environment setting in ENVS, ROUNDS rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rnd in $(seq 1 ${ROUNDS:-2}); do
for E in ${ENVS:-X=0}; do
  env $E timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-queries --no-e2e --cpu-sample 0 $ARGS > gpurun_out/envab.log 2>&1 || { echo "$E failed"; tail -3 gpurun_out/envab.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/envab.log').read().strip().splitlines()[-1]); print('%-22s' % '$E', round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x > 0.01})"
done
done
