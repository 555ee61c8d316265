#!/bin/bash
# Packed-window tokenizer: pack parity tests, then the whole GPU suite, then
# cfg-5-shape and cfg-2 benches (index build only).  Every GPU step bounded.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pack.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_pack.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_pack.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --docs 6250000 --vocab 5000000 --len-min 48 --len-max 80 --cap-log2 23 --steps 3 --warmup 1 --no-queries --no-e2e --cpu-sample 0 > gpurun_out/bench_cfg5.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_cfg5.log; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-queries --no-e2e --cpu-sample 0 > gpurun_out/bench.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.log; exit $rc; }
python3 - <<'PY'
import json
for f in ("gpurun_out/bench_cfg5.log", "gpurun_out/bench.log"):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, "value %.4g docs/s ms/step %.2f pack %s retried %s" % (r["value"], r["ms_per_step"], r.get("tokenizer_docs_per_window"), r.get("pack_retried_docs")))
    print("  phases", {k: round(v, 3) for k, v in r["phases_ms"].items()})
PY
