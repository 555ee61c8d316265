#!/bin/bash
# Unicode path on the GPU box: parity tests, then the build rate of corpora
# with a fraction of non-ASCII documents.  Every GPU step bounded, chained.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_unicode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_uni.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_uni.log; [ $rc -ne 0 ] && exit $rc
for f in ${FRACS:-0.01 0.05 1.0}; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-queries --cpu-sample 0 --no-e2e --unicode-frac $f > gpurun_out/uni_$f.log 2>&1 || exit 1
  python -c "import json; r=json.loads(open('gpurun_out/uni_$f.log').read().strip().splitlines()[-1]); print('$f', r['unicode_docs'], r['long_docs'], round(r['value']/1e6,2), {k: round(v, 3) for k, v in r['phases_ms'].items()})"
done
