#!/bin/bash
# Round-end rehearsal on the GPU box: whole GPU suite, smoke, default bench,
# then the round profile (kernel trace of the bench command + HBM traffic
# passes).  Every GPU step bounded; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -20 gpurun_out/bench.err; exit $rc; }
tail -1 gpurun_out/bench.log
[ -n "${NO_PROF:-}" ] && exit 0
TAG=${TAG:-r01} SQ=${SQ:-} bash tools/prof_round.sh
