#!/bin/bash
# Round 6: the GLOBAL statistics exchange.  (1) one-rank RCCL line (bench.py's
# TFIDF_BENCH_DIST=1 rehearsal); (2) the same under rocprofv3 kernel + HIP API
# trace (bench.py run directly as rank 0 of 1, so the profiler's child is the
# program itself); (3) 8 ranks on the one GPU, collectives over gloo, cfg-3
# shard size (10 M docs / 8 = 1.25 M per rank).
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
A="--steps 10 --warmup 2 --cpu-sample 0 --no-e2e --no-queries"
TFIDF_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py $A > gpurun_out/dist1.json 2> gpurun_out/dist1.err || { tail -5 gpurun_out/dist1.err; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/dist1.json').read().strip().splitlines()[-1]); print('dist1 step %.3f ms exchange %.3f ms' % (r['ms_per_step'], r['global_exchange_ms_per_step']))"
export TMPDIR=/tmp
RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29534 TFIDF_BENCH_DIST=1 \
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d gpurun_out/exch -o exch -- \
  python -u bench.py $A > gpurun_out/dist1_prof.json 2> gpurun_out/dist1_prof.err || { tail -5 gpurun_out/dist1_prof.err; exit 1; }
echo "profiled"
TFIDF_BENCH_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 8 --steps 3 --warmup 1 --docs 1250000 --cpu-sample 0 \
  --no-e2e --no-queries > gpurun_out/gloo8.json 2> gpurun_out/gloo8.err || { tail -5 gpurun_out/gloo8.err; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/gloo8.json').read().strip().splitlines()[-1]); print('gloo8 step %.3f ms exchange %.3f ms' % (r['ms_per_step'], r['global_exchange_ms_per_step']))"
