#!/bin/bash
# Collect rocprofv3 PMC passes for the path kernel (one counter group per pass).
# usage: tools/pmc_passes.sh <outdir> <config> <rows_stride>
set -u
OUT=${1:-gpurun_out/pmc}; CFG=${2:-C2}; STRIDE=${3:-4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for group in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_FLAT" \
             "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --kernel-trace -T -d $OUT/p$i -o p$i --output-format csv -- python3 tools/prof_run.py $CFG 1 $STRIDE > $OUT/p$i.log 2>&1 || echo "pass $i failed rc=$?" >> $OUT/fail.log
done
