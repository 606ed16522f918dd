#!/bin/bash
# r06 call 2: the C4 bench-kernel mismatch diagnosed (records / films, with and
# without records, with and without the tile decomposition), the packed-math
# VALU calibration, and the stall-attribution SQ passes of C2-C5.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c2
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
timeout -k 10 300 python -u tools/diag_bench_kernel.py C4 299 6 > $O/diag_C4.log 2>&1; stop $? diag
timeout -k 10 180 mitsuba0.6_amd/_build/valu_calib > $O/valu_calib.log 2>&1; stop $? calib
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
    SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $O/calib_SQ -o pmc \
    --output-format csv -- mitsuba0.6_amd/_build/valu_calib > $O/calib_SQ.log 2>&1; stop $? calib_sq
for cfg in C2 C3 C4 C5; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU \
      SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --kernel-trace -d $O/stall_${cfg}_A -o pmc \
      --output-format csv -- python3 tools/prof_run.py $cfg 1 4 > $O/stall_${cfg}_A.log 2>&1; stop $? stallA_$cfg
  timeout -s KILL 120 rocprofv3 --pmc VmemLatency SQ_WAVE_CYCLES --kernel-trace -d $O/stall_${cfg}_B -o pmc \
      --output-format csv -- python3 tools/prof_run.py $cfg 1 4 > $O/stall_${cfg}_B.log 2>&1; stop $? stallB_$cfg
  timeout -s KILL 120 rocprofv3 --pmc SmemLatency LdsLatency --kernel-trace -d $O/stall_${cfg}_C -o pmc \
      --output-format csv -- python3 tools/prof_run.py $cfg 1 4 > $O/stall_${cfg}_C.log 2>&1; stop $? stallC_$cfg
done
echo done >> $O/status
