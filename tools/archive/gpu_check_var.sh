#!/bin/bash
# Whole GPU suite, then in-tree lib vs tools/archive/variants/*.so (cfg 2 build), then
# the cfg-5-shape build.  Every GPU step bounded; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/archive/variant_bench.sh || exit 1
timeout -k 10 300 python -u bench.py --docs 6250000 --vocab 5000000 --len-min 48 --len-max 80 --cap-log2 23 --steps 3 --warmup 1 --no-queries --no-e2e --cpu-sample 0 > gpurun_out/bench_cfg5.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_cfg5.log; exit $rc; }
python3 -c "import json; r=json.loads(open('gpurun_out/bench_cfg5.log').read().strip().splitlines()[-1]); print('cfg5 %.4g docs/s' % r['value'], {k: round(v, 3) for k, v in r['phases_ms'].items()})"
