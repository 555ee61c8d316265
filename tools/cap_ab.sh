#!/bin/bash
# cfg-2 build step at the default dictionary size and at 2^20 slots, interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for round in 1 2; do
  echo "== default (2^19)"; bash tools/bench_brief.sh || exit 1
  echo "== 2^20"; bash tools/bench_brief.sh --cap-log2 20 || exit 1
done
