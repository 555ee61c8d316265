#!/bin/bash
# Dictionary capacity sweep: cfg-5 shape at 2^23 / 2^24 slots, cfg 2 at 2^18 / 2^19.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rnd in 1 2; do
for c in ${C5CAPS:-23 24}; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000 --cap-log2 $c --no-queries --no-e2e --cpu-sample 0 > gpurun_out/cap.log 2>&1 || { echo "cfg5 $c failed"; tail -3 gpurun_out/cap.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/cap.log').read().strip().splitlines()[-1]); print('cfg5 cap $c', round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x > 0.01})"
done
for c in ${C2CAPS:-18 19}; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cap-log2 $c --no-queries --no-e2e --cpu-sample 0 > gpurun_out/cap.log 2>&1 || { echo "cfg2 $c failed"; tail -3 gpurun_out/cap.log; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/cap.log').read().strip().splitlines()[-1]); print('cfg2 cap $c', round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x > 0.01})"
done
done
