#!/bin/bash
# Node-level C ABI on the GPU: node / RCCL / multi-rank tests, then the bench's
# multi-GPU code path at one rank (built-in RCCL communicator).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_node.py tests/test_gpu_multirank.py} > gpurun_out/node_tests.log 2>&1
rc=$?; tail -15 gpurun_out/node_tests.log; [ $rc -ne 0 ] && exit $rc
[ -n "$NOBENCH" ] && exit 0
TFIDF_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-e2e > gpurun_out/node_bench.log 2>&1
rc=$?; tail -c 1500 gpurun_out/node_bench.log; exit $rc
