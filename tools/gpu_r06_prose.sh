#!/bin/bash
# Round 6: prose parity (UNI wave rules extended to real typography), then
# build benches: cfg 2 ASCII / prose (UNI on / off), 300 books ASCII / prose.
set -o pipefail
export TFIDF_DEBUG=1   # the library reads its TFIDF_* knobs only under TFIDF_DEBUG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_uni_wave.py tests/test_gpu_unicode.py tests/test_gpu_unicode_sparse.py -x -q --timeout 300 --timeout-method thread > gpurun_out/prose_tests.log 2>&1
rc=$?; tail -6 gpurun_out/prose_tests.log; [ $rc -ne 0 ] && exit $rc
B="python -u bench.py --steps 10 --warmup 2 --no-queries --no-e2e --cpu-sample 0"
line() { python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); ph=r['phases_ms']; print(sys.argv[2], 'step %.3f ms  ' % r['ms_per_step'] + '  '.join('%s %.3f' % (k[3:], v) for k, v in ph.items() if v > 0.001))" $1 $2; }
timeout -k 10 300 $B > gpurun_out/p_ascii.json 2>gpurun_out/p.err && line gpurun_out/p_ascii.json ascii &&
timeout -k 10 300 $B --prose 1 > gpurun_out/p_prose.json 2>>gpurun_out/p.err && line gpurun_out/p_prose.json prose &&
TFIDF_NO_UNIWAVE=1 timeout -k 10 300 $B --prose 1 > gpurun_out/p_prose_nouw.json 2>>gpurun_out/p.err && line gpurun_out/p_prose_nouw.json prose_uwave_only &&
timeout -k 10 300 $B --docs 300 --len-min 80000 --len-max 120000 > gpurun_out/p_books.json 2>>gpurun_out/p.err && line gpurun_out/p_books.json books &&
timeout -k 10 300 $B --docs 300 --len-min 80000 --len-max 120000 --prose 1 > gpurun_out/p_books_prose.json 2>>gpurun_out/p.err && line gpurun_out/p_books_prose.json books_prose
rc=$?; [ $rc -ne 0 ] && tail -5 gpurun_out/p.err; exit $rc
