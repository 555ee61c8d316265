#!/bin/bash
# Run the given pytest selection against each library variant in turn:
# LIBS="base lanemask" bash tools/lib_tests.sh tests/x.py::test_y ...
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out lib_var/base
cp tf-idf-distributed-system_amd/lib/libtfidf.so lib_var/base/libtfidf.so
for v in $LIBS; do
  cp lib_var/$v/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
  timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 200 --timeout-method thread > gpurun_out/lt_$v.log 2>&1
  echo "== $v rc=$?"; tail -3 gpurun_out/lt_$v.log
done
cp lib_var/base/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
