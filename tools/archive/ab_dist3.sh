#!/bin/bash
# The gpu_full.sh one-rank RCCL command (3 steps, warmup 1), side vs main commit tail.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
port=29571
for v in side main side main; do
  if [ $v = main ]; then export TFIDF_MIRROR_MAIN=1; else unset TFIDF_MIRROR_MAIN; fi
  port=$((port+1))
  TFIDF_BENCH_DIST=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --steps 3 --warmup 1 --cpu-sample 0 --no-e2e --batch-queries 2000 > gpurun_out/abd3_$v.log 2> gpurun_out/abd3_$v.err || { tail -5 gpurun_out/abd3_$v.err; exit 1; }
  python3 -c "
import json
r=json.loads(open('gpurun_out/abd3_$v.log').read().strip().splitlines()[-1]); print('$v ms/step %.3f total %.3f exch %.3f' % (r['ms_per_step'], r['phases_ms']['ms_total'], r.get('global_exchange_ms_per_step') or -1))"
done
