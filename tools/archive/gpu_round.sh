#!/bin/bash
# One GPU call: parity tests (TESTS, default all), variant A/B bench, per-phase counters (PHASES=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ "${TESTS:-tests}" != none ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests} > gpurun_out/rt_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/rt_tests.log; [ $rc -ne 0 ] && { grep -E "Error|error|assert" gpurun_out/rt_tests.log | head -30; exit $rc; }
fi
bash tools/archive/variant_bench.sh || exit $?
[ -n "$PHASES" ] && { bash tools/archive/gpu_phases_ab.sh || exit $?; }
exit 0
