#!/bin/bash
# cfg-2 build step per library variant (lib_var/<name>/libtfidf.so; base = the tree's), interleaved.
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p lib_var/base
cp tf-idf-distributed-system_amd/lib/libtfidf.so lib_var/base/libtfidf.so
rc=0
for v in $VARIANTS; do
  cp lib_var/$v/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
  echo "== $v"; bash tools/bench_brief.sh --steps 20 --warmup 3 || { rc=1; break; }
done
cp lib_var/base/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
exit $rc
