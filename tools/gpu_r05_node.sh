#!/bin/bash
# Round 5: process model (1) bench — one process owns the node's GPUs through
# tfidf_node (TFIDF_BENCH_NODE=1); on the 1-GPU box, a node of one shard.
set -o pipefail
mkdir -p gpurun_out
TFIDF_BENCH_NODE=1 timeout -k 10 300 python -u bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench_node1.log 2> gpurun_out/bench_node1.err
rc=$?; tail -3 gpurun_out/bench_node1.err; tail -1 gpurun_out/bench_node1.log; exit $rc
