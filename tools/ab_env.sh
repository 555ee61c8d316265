#!/bin/bash
# A/B of environment settings on the cfg-2 build bench (tools/bench_brief.sh):
# SETS is a ';'-separated list of settings ("" = defaults), each run twice,
# interleaved.  Example: SETS='; TFIDF_SORT_SPW=2; TFIDF_SORT_THREADS=1024'.
# CMD: the measurement (default: the build bench).
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
CMD=${CMD:-"bash tools/bench_brief.sh"}
IFS=';' read -ra LIST <<< "$SETS"
for round in 1 2; do
  for s in "${LIST[@]}"; do
    echo "== [${s}] (round $round)"
    env $s timeout -k 10 240 $CMD 2>&1 | tail -${TAILN:-1} || exit 1
  done
done
