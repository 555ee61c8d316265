#!/bin/bash
# The whole -m gpu suite (bounded), then smoke().  Extra arguments go to pytest.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --durations=10 --timeout 300 --timeout-method thread "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -16 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; exit $rc
