#!/bin/bash
# Round-2 profile refresh at the final kernels: kernel trace + PMC traffic +
# SQ counters of the default bench (prof_round.sh), then the tokenizer
# per-phase counters (prof_phases.sh).  Every GPU step bounded inside.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=r02 SQ=1 bash tools/prof_round.sh > gpurun_out/prof_round.log 2>&1 || { tail -20 gpurun_out/prof_round.log; exit 1; }
echo "prof_round ok"
cd $R && STOPS="1 2 3 4 0" bash tools/prof_phases.sh > gpurun_out/prof_phases.log 2>&1 || { tail -20 gpurun_out/prof_phases.log; exit 2; }
echo "prof_phases ok"
