#!/bin/bash
# r04: PMC passes over the wavefront engine on C4 (1/4 of the rows): the SQ
# wave-cycle budget, then HBM FETCH/WRITE, per dispatch (tools/wf_pmc_summary.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_wfpmc
mkdir -p $O
for c in ${CFGS:-C4}; do
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/sq_$c -o pmc --output-format csv \
    -- python3 tools/prof_run.py $c 1 4 wavefront > $O/sq_$c.log 2>&1 || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace -d $O/${ctr}_$c -o pmc --output-format csv \
    -- python3 tools/prof_run.py $c 1 4 wavefront > $O/${ctr}_$c.log 2>&1 || exit 1
done
done
