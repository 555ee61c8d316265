#!/bin/bash
# GPU tests (optional), then the variant A/B bench (tools/archive/variant_bench.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $TESTS > gpurun_out/ab_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && { grep -E "Error|error|assert" gpurun_out/ab_tests.log | head -30; exit $rc; }
fi
bash tools/archive/variant_bench.sh
