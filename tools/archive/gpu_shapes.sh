#!/bin/bash
# Bench lines of the other BASELINE shapes: cfg 5 per-GPU share (6.25 M short
# docs, V = 5 M) and cfg 1 (300 book-sized documents).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --docs 6250000 --vocab 5000000 --len-min 48 --len-max 80 --steps 3 --warmup 1 --no-queries --cpu-sample 0 --no-e2e > gpurun_out/bench_cfg5.log 2> gpurun_out/bench_cfg5.err || { tail -5 gpurun_out/bench_cfg5.err; exit 1; }
timeout -k 10 300 python -u bench.py --docs 300 --len-min 80000 --len-max 120000 --steps 5 --warmup 2 --cpu-sample 40 --no-e2e --batch-queries 1000 > gpurun_out/bench_book.log 2> gpurun_out/bench_book.err || { tail -5 gpurun_out/bench_book.err; exit 2; }
python - <<'PY'
import json
for f in ("gpurun_out/bench_cfg5.log", "gpurun_out/bench_book.log"):
    r = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, "value %.4g docs/s ms/step %.2f" % (r["value"], r["ms_per_step"]), {k: round(v, 3) for k, v in r["phases_ms"].items()}, r["roofline"]["kernel"], round(r["roofline"]["frac"], 4))
PY
