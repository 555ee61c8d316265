#!/bin/bash
# Cost of the UNI prose check in the full pipeline: lib_var/check2 runs it twice
# at TFIDF_DEBUG_STOP=8 (the second pass over its own output); stop 9 = once.
set -o pipefail
export TFIDF_DEBUG=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p lib_var/base gpurun_out
cp tf-idf-distributed-system_amd/lib/libtfidf.so lib_var/base/libtfidf.so
cp lib_var/check2/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
for st in 9 8 9 8; do
  TFIDF_DEBUG_STOP=$st timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-queries --cpu-sample 0 --no-e2e --prose 1 > gpurun_out/pc_$st.log 2>gpurun_out/pc.err || { tail -3 gpurun_out/pc.err; break; }
  python3 -c "import json; r=json.loads(open('gpurun_out/pc_$st.log').read().strip().splitlines()[-1]); print('stop $st tokenize %.3f' % r['phases_ms']['ms_tokenize'])"
done
cp lib_var/base/libtfidf.so tf-idf-distributed-system_amd/lib/libtfidf.so
