#!/bin/bash
# r04: roughplastic's warped alpha once per vertex (RpPre::walpha) -- A/B against
# the previous build on C5 (megakernel and wavefront), C3 as the control
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
B=mitsuba0.6_amd/_build/variants/libmtsgpu_base.so
N=mitsuba0.6_amd/_build/variants/libmtsgpu_rpw.so
for c in C5 C3; do echo "== $c" >> gpurun_out/r04_ab_rpw.log; timeout -k 10 300 python -u tools/ab_variants.py $c 4 4 base=$B rpw=$N >> gpurun_out/r04_ab_rpw.log 2>&1 || exit 1; done
echo "== C5 wavefront" >> gpurun_out/r04_ab_rpw.log
AB_ENGINE=wavefront timeout -k 10 300 python -u tools/ab_variants.py C5 3 4 base=$B rpw=$N >> gpurun_out/r04_ab_rpw.log 2>&1 || exit 1
