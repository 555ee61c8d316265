#!/bin/bash
# 2-rank rehearsal of bench.py's multi-GPU path on a 1-GPU box: both ranks on
# cuda:0, collectives over gloo (RCCL needs one GPU per rank).
set -o pipefail
mkdir -p gpurun_out
TFIDF_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --docs ${DOCS:-200000} \
  --cpu-sample 0 > gpurun_out/multi.log 2>&1
rc=$?; tail -3 gpurun_out/multi.log | cut -c1-600; exit $rc
