set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rocprofv3 -L > $R/gpurun_out/prof/counters_list.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/kt -o kt --output-format csv -- python3 $R/bench.py --docs 200000 --steps 2 --warmup 1 --no-queries --cpu-sample 0 > $R/gpurun_out/prof/kt_bench.log 2>&1
echo kt rc=$?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --kernel-include-regex tokenize -d $R/gpurun_out/prof/pmc1 -o pmc1 --output-format csv -- python3 $R/bench.py --docs 200000 --steps 1 --warmup 0 --no-queries --cpu-sample 0 > $R/gpurun_out/prof/pmc1_bench.log 2>&1
echo pmc1 rc=$?
