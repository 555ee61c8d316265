#!/bin/bash
# round 3: new multi-rank / coalescing tests, then the full-size 8-shard tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 380 --timeout-method thread \
  tests/test_gpu_multirank.py tests/test_gpu_operators.py -k "coalesce or multirank or seed" \
  > gpurun_out/r03a_t1.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 420 --timeout-method thread \
  tests/test_gpu_fullsize_multirank.py > gpurun_out/r03a_t2.log 2>&1
