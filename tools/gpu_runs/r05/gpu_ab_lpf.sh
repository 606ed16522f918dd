#!/bin/bash
# r05: BVH leaf loop with the next record's loads in flight during the current test (MTSG_LEAF_PREFETCH)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_lpf.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 cur=$L lpf=$V/libmtsgpu_lpf.so >> gpurun_out/r05_ab_lpf.log 2>&1 || exit 1; done
