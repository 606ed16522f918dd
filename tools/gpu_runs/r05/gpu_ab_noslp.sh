#!/bin/bash
# r05: ray origin = P.its.p and double constants materialised in place (rokd), then
# the same without the SLP vectoriser (noslp), vs the committed slim build
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
V=mitsuba0.6_amd/_build/variants
for c in C2 C3 C4 C5; do echo "== $c" >> gpurun_out/r05_ab_noslp.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 slim=$V/libmtsgpu_slim.so rokd=$V/libmtsgpu_rokd.so noslp=$V/libmtsgpu_noslp.so >> gpurun_out/r05_ab_noslp.log 2>&1 || exit 1; done
for c in C3 C4 C5; do echo "== wavefront $c" >> gpurun_out/r05_ab_noslp.log; timeout -k 10 300 python -u tools/ab_variants.py $c 2 4 slim=$V/libmtsgpu_slim.so,ENGINE=wavefront noslp=$V/libmtsgpu_noslp.so,ENGINE=wavefront >> gpurun_out/r05_ab_noslp.log 2>&1 || exit 1; done
