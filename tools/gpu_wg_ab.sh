#!/bin/bash
# Workgroup tokenizer: parity tests on the in-tree build, then cfg-2 bench A/B:
# in-tree (k_tokenize_wg), the wave kernel (TFIDF_TOK_WAVE=1), tools/variants/*.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ "${TESTS:-x}" != none ]; then
  TFIDF_TOK_WG=1 timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_identity.py tests/test_gpu_unicode.py tests/test_gpu_pack.py} > gpurun_out/wg_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/wg_tests.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/wg_tests.log | head -30; exit $rc; }
fi
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
run() {  # name, env
  env $2 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-queries --no-e2e --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/wg.log 2>&1 || { echo "$1 failed"; tail -3 gpurun_out/wg.log; cp /tmp/libtfidf_base.so $L; exit 1; }
  python3 -c "import json; r=json.loads(open('gpurun_out/wg.log').read().strip().splitlines()[-1]); print('%-24s' % '$1', round(r['ms_per_step'], 3), {k: round(x, 3) for k, x in r['phases_ms'].items() if x})"
}
for rnd in $(seq 1 ${ROUNDS:-2}); do
  cp /tmp/libtfidf_base.so $L; run wg TFIDF_TOK_WG=1; run wave X=1
  for v in tools/variants/*.so; do [ -e "$v" ] || continue; cp $v $L; run $(basename $v) TFIDF_TOK_WG=1; done
done
cp /tmp/libtfidf_base.so $L
