#!/bin/bash
# r05: BVH nodes in treelet order (128-byte lines: node, children, first grandchild) vs depth-first order
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
T=mitsuba0.6_amd/_build/variants/libmtsgpu_treelet.so
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_treelet.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 dfs=$L treelet=$T >> gpurun_out/r05_ab_treelet.log 2>&1 || exit 1; done
