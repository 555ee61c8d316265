#!/bin/bash
# Round 5 check: parity subset, then cfg 2 (ASCII, 100 % / 10 % non-ASCII) and
# the cfg-5 shape (packed windows) bench lines at the current code.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_uni_wave.py tests/test_gpu_pack.py tests/test_gpu_parity.py tests/test_gpu_unicode.py > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/ab_tests.log | head -20; exit $rc; }
run() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > gpurun_out/ab_$n.log 2> gpurun_out/ab_$n.err || { echo "$n failed"; tail -5 gpurun_out/ab_$n.err; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/ab_$n.log').read().strip().splitlines()[-1]); print('$n', round(r['ms_per_step'], 3), 'ms/step, tokenize', round(r['phases_ms']['ms_tokenize'], 3))"
}
run ascii 200 --steps 10 --warmup 2 --no-queries --no-e2e --cpu-sample 0
run uni100 200 --steps 5 --warmup 2 --unicode-frac 1.0 --no-queries --no-e2e --cpu-sample 0
run uni10 200 --steps 5 --warmup 2 --unicode-frac 0.1 --no-queries --no-e2e --cpu-sample 0
run cfg5 300 --steps 5 --warmup 2 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000 --no-queries --no-e2e --cpu-sample 0
run ascii2 200 --steps 10 --warmup 2 --no-queries --no-e2e --cpu-sample 0
