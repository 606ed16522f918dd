#!/bin/bash
# Round profiling on the GPU box (run through gpurun from the repo root):
#  1. rocprofv3 --kernel-trace --stats of the bench command itself (C2, C3)
#  2. separate PMC passes FETCH_SIZE / WRITE_SIZE (MI355X_MICROARCH.md "HBM")
#     over one full frame of each config, for bench.py's roofline.traffic
#  3. one SQ pass (wave cycles, VALU issue, waits) for bench.py's roofline.valu
#  4. three stall-attribution passes (instruction kinds, VMEM / SMEM / LDS latency)
# Every GPU step has its own time limit; the script stops at the first failure.
set -eu
OUT=${1:-gpurun_out/prof}
ROOT=$(pwd)
mkdir -p $OUT
export TMPDIR=/tmp
# the 1/4-row SQ and stall passes run the full frame's sample-run length (tools/prof_run.py)
export PROF_FULL_RUNS=1
# the build these profiles describe (bench.py only trusts profiles of the library it times)
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so | cut -d' ' -f1 > $OUT/lib.sha256
for cfg in ${CONFIGS:-C2 C3 C4 C5 C2g}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench_$cfg -o bench --output-format csv \
      -- python3 $ROOT/bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --secondary none > $OUT/bench_$cfg.log 2>&1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -d $OUT/pmc_${cfg}_$ctr -o pmc --output-format csv \
        -- python3 $ROOT/tools/prof_run.py $cfg 1 1 > $OUT/pmc_${cfg}_$ctr.log 2>&1
  done
  # wave-cycle budget (VALU issue, waits) over 1/4 of the rows: 8 SQ counters + 1 GRBM
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc_${cfg}_SQ -o pmc \
      --output-format csv -- python3 $ROOT/tools/prof_run.py $cfg 1 4 > $OUT/pmc_${cfg}_SQ.log 2>&1
  # stall attribution (tools/stall_summary.py): instruction counts by kind, and VMEM / SMEM / LDS latencies
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU \
      SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace -d $OUT/stall_${cfg}_A -o pmc \
      --output-format csv -- python3 $ROOT/tools/prof_run.py $cfg 1 4 > $OUT/stall_${cfg}_A.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc VmemLatency SQ_WAVE_CYCLES --kernel-trace -d $OUT/stall_${cfg}_B -o pmc \
      --output-format csv -- python3 $ROOT/tools/prof_run.py $cfg 1 4 > $OUT/stall_${cfg}_B.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SmemLatency LdsLatency --kernel-trace -d $OUT/stall_${cfg}_C -o pmc \
      --output-format csv -- python3 $ROOT/tools/prof_run.py $cfg 1 4 > $OUT/stall_${cfg}_C.log 2>&1
done
echo done > $OUT/ok
