#!/bin/bash
# r05: the GVN-PRE defect on today's source: the shipped build (PRE off) and the PRE-on build of
# path_kernel.hip (tools/gpu_runs/r05/gvn_pre_repro.sh) against the oracle on the direct-integrator scenes
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/diag_parity.py --only=direct_shapes,indep_direct_shapes,direct_env \
    preon=mitsuba0.6_amd/_build/variants/libmtsgpu_preon.so > gpurun_out/r05_gvn_pre_repro.log 2>&1
