#!/bin/bash
# 10 k-query batch device time (tools/time_batch_host.py) per environment
# setting in ENVS, ROUNDS rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
for rnd in $(seq 1 ${ROUNDS:-2}); do
for E in ${ENVS:-X=0}; do
  env $E timeout -k 10 300 python3 tools/time_batch_host.py > gpurun_out/be.log 2>&1 || { echo "$E failed"; tail -3 gpurun_out/be.log; exit 1; }
  echo "$E: $(grep -E 'device' gpurun_out/be.log | tail -1)"
done
done
