#!/bin/bash
# r06 call 1: the bench kernels against the oracle + RCCL at world size 1 (new tests),
# the counter list, and the VALU calibration kernel (plain timing + one SQ pass).
# A GPU fault / abort / time limit ends the script; a failing test does not.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c1
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
MTSGPU_TEST_LOGDIR=$O timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_bench_kernels.py tests/test_gpu_rccl.py > $O/tests.log 2>&1; stop $? tests
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; stop $? counters
timeout -k 10 120 mitsuba0.6_amd/_build/valu_calib > $O/valu_calib.log 2>&1; stop $? calib
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
    SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace -d $O/calib_SQ -o pmc \
    --output-format csv -- mitsuba0.6_amd/_build/valu_calib > $O/calib_SQ.log 2>&1; stop $? calib_sq
echo done >> $O/status
