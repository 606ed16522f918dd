#!/bin/bash
# r05: existing knobs re-measured on the slimmer kernels: C2 through its BVH instead of
# the 32-triangle scan; large scenes with fewer Sobol dimensions in LDS
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
echo "== C2" >> gpurun_out/r05_ab_knobs.log; timeout -k 10 300 python -u tools/ab_variants.py C2 3 4 scan=$L bvh=$L,MTSGPU_NO_SCAN=1 >> gpurun_out/r05_ab_knobs.log 2>&1 || exit 1
for c in C3 C4; do echo "== $c" >> gpurun_out/r05_ab_knobs.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 dflt=$L dims4=$L,MTSGPU_SOBOL_LDS_DIMS=4 dims0=$L,MTSGPU_SOBOL_LDS_DIMS=0 >> gpurun_out/r05_ab_knobs.log 2>&1 || exit 1; done
