#!/bin/bash
# r05: a bounce's shadow and closest-hit rays through the BVH in one joint traversal (traverse_pair, round 3) at today's register pressure
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/variants/libmtsgpu_base.so
T=mitsuba0.6_amd/_build/variants/libmtsgpu_pair.so
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_pair.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 base=$L pair=$T >> gpurun_out/r05_ab_pair.log 2>&1 || exit 1; done
