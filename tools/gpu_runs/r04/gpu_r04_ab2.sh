#!/bin/bash
# r04: per-kernel profile of the wavefront engine (C3-C5), then A/B of the
# shade kernels' LDS Sobol staging
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
TAG=r04_wfprof2 bash tools/gpu_wf_prof.sh || exit 1
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C3 C4 C5; do echo "== $c" >> gpurun_out/r04_ab2.log; timeout -k 10 240 python -u tools/ab_variants.py $c 3 4 wave=$L,ENGINE=wavefront wave_nolds=$L,ENGINE=wavefront,MTSGPU_WF_SHADE_LDS_DIMS=0 >> gpurun_out/r04_ab2.log 2>&1 || exit 1; done
