set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_identity.py tests/test_gpu_pack.py tests/test_gpu_books.py tests/test_gpu_term_major.py tests/test_gpu_fullsize.py > gpurun_out/g4_tests.log 2>&1 || { tail -30 gpurun_out/g4_tests.log; exit 1; }
tail -2 gpurun_out/g4_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-queries --cpu-sample 0 --no-e2e > gpurun_out/g4_cfg2.log 2>gpurun_out/g4_cfg2.err || exit 2
bash tools/archive/gpu_shapes.sh
python -c "
import json;r=json.loads(open('gpurun_out/g4_cfg2.log').read().strip().splitlines()[-1]);print('cfg2',r['value'],r['ms_per_step'],r['phases_ms'])"
