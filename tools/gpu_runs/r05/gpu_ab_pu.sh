#!/bin/bash
# r05: the leaf loop reading the next record unconditionally (padding record after the last) against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_leaf_uncond.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 head=$V/libmtsgpu_head.so uncond=$V/libmtsgpu_pu.so >> gpurun_out/r05_ab_leaf_uncond.log 2>&1 || exit 1; done
