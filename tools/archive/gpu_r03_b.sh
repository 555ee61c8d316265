#!/bin/bash
# whole GPU suite, then the tokenizer's per-phase SQ counters (tools/prof_phases.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/gpu_tests.log | head -30; exit $rc; }
STOPS="1 2 3 4 0" bash tools/prof_phases.sh > gpurun_out/phases.txt 2>&1; rc=$?; cat gpurun_out/phases.txt; exit $rc
