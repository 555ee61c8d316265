#!/bin/bash
# One cfg-2 bench line (no queries), printed as step / phase times.  Extra
# arguments go to bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
python -u bench.py --steps 10 --warmup 2 --no-queries --no-e2e --cpu-sample 0 "$@" > gpurun_out/brief.json 2> gpurun_out/brief.err || { tail -5 gpurun_out/brief.err; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/brief.json').read().strip().splitlines()[-1]); ph=r['phases_ms']; print('step %.3f ms  ' % r['ms_per_step'] + '  '.join('%s %.3f' % (k[3:], v) for k, v in ph.items() if v > 0.001))"
