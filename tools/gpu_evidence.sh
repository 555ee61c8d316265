#!/bin/bash
# Round evidence at the current code (GPU box): kernel trace + PMC traffic +
# SQ counters of the default bench (tools/prof_round.sh), then the bench lines
# the docs cite: default (cfg 2, with queries, end-to-end and the CPU
# baseline; roofline.traffic from this run's PMC pass), cfg-5 shape, 300-book
# shape, books with one non-ASCII word per ~2 KB (chunk path, and with the
# Unicode chunk path disabled), cfg 2 with 10 % / all documents non-ASCII,
# the cfg-5 PMC summary, and the one-rank RCCL
# rehearsal of the node path.  Output: gpurun_out/ev_$TAG/.
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${TAG:-r06}; O=$R/gpurun_out/ev_$TAG; mkdir -p $O
TAG=$TAG SQ=1 bash tools/prof_round.sh > $O/prof_round.log 2>&1 || { echo "prof_round failed"; tail -5 $O/prof_round.log; exit 1; }
tail -3 $O/prof_round.log
TJ=$R/gpurun_out/prof_$TAG/traffic.json
run() {   # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.log 2> $O/$n.err || { echo "$n failed"; tail -5 $O/$n.err; exit 1; }
  tail -1 $O/$n.log > $O/$n.json
  python3 -c "import json; r=json.load(open('$O/$n.json')); print('$n', round(r['value']/1e6, 2), 'M docs/s', round(r['ms_per_step'], 3), 'ms', {k: round(v, 3) for k, v in r['phases_ms'].items() if v > 0.01})"
}
run bench_line 400 --traffic-json $TJ
run bench_line_cfg5_shape 300 --steps 5 --warmup 2 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000 --no-queries --no-e2e --cpu-sample 0
run bench_line_book_shape 200 --steps 10 --warmup 2 --docs 300 --len-min 80000 --len-max 120000 --no-queries --no-e2e --cpu-sample 0
run bench_line_book_unicode 200 --steps 10 --warmup 2 --docs 300 --len-min 80000 --len-max 120000 --unicode-every 2048 --no-queries --no-e2e --cpu-sample 0
TFIDF_NO_UCHUNK=1 run bench_line_book_unicode_whole_book 200 --steps 10 --warmup 2 --docs 300 --len-min 80000 --len-max 120000 --unicode-every 2048 --no-queries --no-e2e --cpu-sample 0
run bench_line_cfg2_unicode10 200 --steps 5 --warmup 2 --unicode-frac 0.1 --no-queries --no-e2e --cpu-sample 0
run bench_line_cfg2_unicode100 300 --steps 3 --warmup 1 --unicode-frac 1.0 --no-queries --no-e2e --cpu-sample 0
run bench_line_cfg2_prose 300 --steps 10 --warmup 2 --prose 1 --no-queries --no-e2e --cpu-sample 0
TFIDF_NO_UNIFIRST=1 run bench_line_cfg2_prose_ascii_first 300 --steps 10 --warmup 2 --prose 1 --no-queries --no-e2e --cpu-sample 0
TFIDF_NO_UNIWAVE=1 run bench_line_cfg2_prose_uwave_only 300 --steps 5 --warmup 1 --prose 1 --no-queries --no-e2e --cpu-sample 0
TFIDF_BENCH_NODE=1 run bench_line_node1 300 --steps 5 --warmup 2 --cpu-sample 0 --no-e2e
run bench_line_books_prose 200 --steps 10 --warmup 2 --docs 300 --len-min 80000 --len-max 120000 --prose 1 --no-queries --no-e2e --cpu-sample 0
# cfg-5 PMC: one build, FETCH / WRITE passes, kernel summary
P=$R/gpurun_out/prof_cfg5_$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
C5="python3 $R/bench.py --steps 1 --warmup 0 --docs 6250000 --len-min 48 --len-max 80 --vocab 5000000 --no-queries --no-e2e --cpu-sample 0"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $P/kt -o kt --output-format csv -- $C5 > $P/kt.log 2>&1 || { echo "cfg5 kt failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_" -d $P/fetch -o fetch --output-format csv -- $C5 > $P/fetch.log 2>&1 || { echo "cfg5 fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_" -d $P/write -o write --output-format csv -- $C5 > $P/write.log 2>&1 || { echo "cfg5 write failed"; exit 1; }
python3 $R/tools/summarize_prof.py $P --json $P/traffic.json > $P/summary.txt 2>&1 || true
head -12 $P/summary.txt
cd $R
TFIDF_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-e2e --batch-queries 2000 > $O/bench_dist1.log 2> $O/bench_dist1.err || { echo "dist failed"; tail -5 $O/bench_dist1.err; exit 1; }
tail -1 $O/bench_dist1.log > $O/bench_line_dist1_rccl.json
echo "evidence ok"
