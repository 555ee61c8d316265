#!/bin/bash
# WG tokenizer parity (punctuation corpus first), Unicode chunk path, A/B, node tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TFIDF_TOK_WG=1 timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread "tests/test_gpu_parity.py::test_punctuation_corpus_parity" > gpurun_out/wg_p1.log 2>&1
rc=$?; tail -3 gpurun_out/wg_p1.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_unicode.py tests/test_gpu_books.py > gpurun_out/uchunk.log 2>&1
rc=$?; tail -3 gpurun_out/uchunk.log; [ $rc -ne 0 ] && { grep -nE "FAIL|Error|assert" gpurun_out/uchunk.log | head -20; exit $rc; }
TESTS="tests/test_gpu_parity.py tests/test_gpu_identity.py tests/test_gpu_unicode.py tests/test_gpu_pack.py tests/test_gpu_books.py" ROUNDS=1 bash tools/gpu_wg_ab.sh || exit $?
NOBENCH=1 bash tools/archive/gpu_node.sh
