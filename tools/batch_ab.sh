#!/bin/bash
# Batch device time under launch-shape knobs: SETS="name:VAR=val,VAR=val ..."
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for spec in $SETS; do
  n=${spec%%:*}; e=""; [ "$n" != "$spec" ] && e=${spec#*:}
  echo "== $n $e"
  ( [ -n "$e" ] && export ${e//,/ }; bash tools/batch_brief.sh ) || exit 1
done
