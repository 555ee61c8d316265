#!/bin/bash
# Query-unit batch path: its parity tests, then the cfg-4 batch timing A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_units.py -x -v --timeout 120 --timeout-method thread > gpurun_out/units_tests.log 2>&1
rc=$?; tail -12 gpurun_out/units_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/archive/batch_units.py > gpurun_out/batch_units.log 2>&1
rc=$?; cat gpurun_out/batch_units.log | tail -5; exit $rc
