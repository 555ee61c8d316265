#!/bin/bash
# Round profile: rocprofv3 kernel-trace summary of the bench command, HBM
# traffic (FETCH_SIZE / WRITE_SIZE, separate passes) and SQ counters for every
# kernel of one index build, then the tokenize ablation if ABLATE is set.
# Every GPU step bounded.  Usage (GPU box): TAG=r01 bash tools/prof_round.sh
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r01}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py ${BENCH_ARGS:-}"
if [ -z "${NO_KT:-}" ]; then
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $BENCH > $O/kt_bench.log 2>&1 || { echo "kt failed"; tail -5 $O/kt_bench.log; exit 1; }
  echo "kt ok"
fi
SMALL="python3 $R/bench.py --steps 1 --warmup 0 --no-queries --cpu-sample 0 ${PMC_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_" -d $O/fetch -o fetch --output-format csv -- $SMALL > $O/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $O/fetch.log; exit 2; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_" -d $O/write -o write --output-format csv -- $SMALL > $O/write.log 2>&1 || { echo "write failed"; tail -5 $O/write.log; exit 3; }
echo "traffic ok"
grep '"metric"' $O/fetch.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); c=r['config']; json.dump({'docs_per_gpu': c['docs_per_gpu'], 'text_bytes_per_gpu': c['text_bytes_per_gpu'], 'nnz_per_gpu': c['nnz_per_gpu']}, open('$O/workload.json','w'))" || true
if [ -n "${SQ:-}" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "k_" -d $O/sq1 -o sq1 --output-format csv -- $SMALL > $O/sq1.log 2>&1 || { echo "sq1 failed"; exit 4; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES --kernel-include-regex "k_" -d $O/sq2 -o sq2 --output-format csv -- $SMALL > $O/sq2.log 2>&1 || { echo "sq2 failed"; exit 5; }
  echo "sq ok"
fi
if [ -n "${ABLATE:-}" ]; then
  cd $R
  for s in 1 2 3 4 0; do
    TFIDF_DEBUG_STOP=$s timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-queries --cpu-sample 0 > $O/ablate_$s.log 2>&1
    python3 -c "import json; r=json.loads(open('$O/ablate_$s.log').read().strip().splitlines()[-1]); print('stop=$s tokenize_ms=%.3f' % r['phases_ms']['ms_tokenize'])" 2>/dev/null || { echo "stop=$s: no json"; tail -3 $O/ablate_$s.log; }
  done
fi
python3 $R/tools/summarize_prof.py $O --json $O/traffic.json
