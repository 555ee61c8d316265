#!/bin/bash
# Whole GPU suite, smoke, default bench, then the multi-GPU code path over RCCL
# at one rank (TFIDF_BENCH_DIST=1: process group, GLOBAL exchange, node-level
# batched queries).  Every GPU step bounded; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --durations=15 --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
python - <<'PY'
import json
r = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value %.4g docs/s  ms/step %.2f" % (r["value"], r["ms_per_step"]))
print("roofline", {k: r["roofline"][k] for k in ("kernel", "achieved", "frac", "avg_launch_ms")})
print("queries", {k: v for k, v in r.get("queries", {}).items() if k != "roofline"})
PY
[ -n "${NO_DIST:-}" ] && exit 0
TFIDF_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-e2e --batch-queries 2000 > gpurun_out/bench_dist1.log 2> gpurun_out/bench_dist1.err
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench_dist1.err; exit $rc; }
tail -1 gpurun_out/bench_dist1.log | cut -c1-600
