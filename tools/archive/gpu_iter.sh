#!/bin/bash
# Iteration loop on the GPU box: parity tests, then a short bench; every GPU
# step bounded and chained (stop at the first failure).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --cpu-sample ${CPUS:-2000} ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value %.4g docs/s  ms/step %.2f" % (r["value"], r["ms_per_step"]))
print("roofline", {k: r["roofline"][k] for k in ("kernel", "achieved", "frac", "avg_launch_ms")})
print("phases", {k: round(v, 3) for k, v in r["phases_ms"].items()})
print("queries", r.get("queries"))
print("e2e", r.get("end_to_end"), "copyGBs", r["roofline"].get("measured_copy_GBs"))
PY
