#!/bin/bash
# Per-phase SQ counters (tools/prof_phases.sh) for the in-tree library and each tools/archive/variants/*.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
L=tf-idf-distributed-system_amd/lib/libtfidf.so
cp $L /tmp/libtfidf_base.so
for v in base ${VARIANTS:-tools/archive/variants/*.so}; do
  n=$(basename $v .so)
  if [ "$v" = base ]; then cp /tmp/libtfidf_base.so $L; else cp $v $L; fi
  rm -rf gpurun_out/prof_phases
  STOPS="${STOPS:-2 3 4 0}" DOCS=${DOCS:-200000} bash tools/prof_phases.sh > gpurun_out/phases_$n.txt 2>&1 || { echo "$n failed"; tail -5 gpurun_out/phases_$n.txt; cp /tmp/libtfidf_base.so $L; exit 1; }
  echo "== $n"; grep -E "SQ_INSTS_VALU|SQ_INSTS_LDS|SQ_WAVE_CYCLES|SQ_WAIT_ANY|SQ_LDS_BANK|SQ_LDS_IDX|SQ_INSTS_SALU|SQ_ACTIVE_INST_VALU" gpurun_out/phases_$n.txt
done
cp /tmp/libtfidf_base.so $L
