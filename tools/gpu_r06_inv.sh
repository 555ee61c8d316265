#!/bin/bash
# Round 6: count-free inversion — parity (inversion tests), kernel traces of
# this tree's library against lib_var/cols (column inversion, two CSR reads),
# then the prose script.
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_inversion_shapes.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/inv_tests.log 2>&1
rc=$?; tail -8 gpurun_out/inv_tests.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base cols base" bash tools/kt_ab.sh || exit $?
bash tools/bench_brief.sh || exit $?
[ -n "$NO_PROSE" ] || bash tools/gpu_r06_prose.sh
