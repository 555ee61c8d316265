#!/bin/bash
# Split wave path A/B: TFIDF_SPLIT=1 (k_tokenize_wave<SPLIT> stages each unit's
# distinct terms, k_resolve_wave resolves them and writes the rows) against
# the fused k_tokenize_wave.  Parity TESTS run on the split path first, then
# the bench SHAPES for both forms, ROUNDS times, then one kernel trace of the
# split form at cfg 2 (per-kernel durations).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TFIDF_SPLIT=1
[ -n "$TRACE_ONLY" ] || {
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread $TESTS > gpurun_out/split_tests.log 2>&1
rc=$?; echo "split tests: $(tail -1 gpurun_out/split_tests.log)"
[ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/split_tests.log | head -30; exit $rc; }
for rnd in $(seq 1 ${ROUNDS:-2}); do
for sp in 0 1; do
  export TFIDF_SPLIT=$sp
  for shape in ${SHAPES:-cfg2}; do
    A="--steps 5 --warmup 2"
    [ $shape = cfg5 ] && A="--steps 3 --warmup 1 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000"
    [ $shape = book ] && A="--steps 5 --warmup 2 --docs 300 --len-min 80000 --len-max 120000"
    timeout -k 10 300 python -u bench.py $A --no-queries --no-e2e --cpu-sample 0 > gpurun_out/tok.log 2>&1 || { echo "split=$sp $shape failed"; tail -3 gpurun_out/tok.log; exit 1; }
    python3 -c "import json; r=json.loads(open('gpurun_out/tok.log').read().strip().splitlines()[-1]); print('split=%s %-6s' % ('$sp', '$shape'), round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x > 0.01})"
  done
done
done
}
export TFIDF_SPLIT=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_split -o split --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-queries --no-e2e --cpu-sample 0 > $R/gpurun_out/prof_split.log 2>&1 || { echo "trace failed"; tail -3 $R/gpurun_out/prof_split.log; exit 1; }
f=$(find $R/gpurun_out/prof_split -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print("%-60s calls %5s avg %.3f ms total %.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
EOF
