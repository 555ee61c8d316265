#!/bin/bash
# Batch timing per library variant (lib_var/<name>/libtfidf.so; base = the tree's):
# VARIANTS="name[:VAR=val,...] ..."
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p lib_var/base
cp tf-idf-distributed-system_amd/lib/libtfidf.so lib_var/base/libtfidf.so
rc=0
for spec in $VARIANTS; do
  v=${spec%%:*}; e=""; [ "$v" != "$spec" ] && e=${spec#*:}
  cp lib_var/$v/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
  echo "== $v $e"
  ( [ -n "$e" ] && export ${e//,/ }; bash tools/batch_brief.sh ) || { rc=1; break; }
done
cp lib_var/base/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
exit $rc
