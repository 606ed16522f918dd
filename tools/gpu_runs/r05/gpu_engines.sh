#!/bin/bash
# r05: the three engines on today's build: megakernel (BVH), wavefront (BVH), kd-tree (wavefront, reference tie order)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C3 C4; do echo "== $c (1/16 of the rows)" >> gpurun_out/r05_engines.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 16 mega=$L,ENGINE=megakernel wave=$L,ENGINE=wavefront kd=$L,ENGINE=kdtree >> gpurun_out/r05_engines.log 2>&1 || exit 1; done
