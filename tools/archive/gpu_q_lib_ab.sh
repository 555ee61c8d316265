#!/bin/bash
# Query-section A/B of tools/archive/variants/*.so against the in-tree library (all hits and single top-10)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
for rnd in 1 2; do
for v in base tools/archive/variants/*.so; do
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --cpu-sample 0 --no-e2e > gpurun_out/qlib.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/qlib.log; cp /tmp/libtfidf_base.so $L; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/qlib.log').read().strip().splitlines()[-1]); q=r['queries']; print('%-26s' % '$v', {k: round(q[k], 4) for k in ('single_all_hits_qps','single_all_hits_device_ms_avg','single_top10_p50_ms')})"
done
done
cp /tmp/libtfidf_base.so $L
