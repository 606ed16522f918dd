#!/bin/bash
# r05: the closest hit's primitive index returned by the traversal instead of reloaded from tris[slot] (prim), plus vertex normals loaded beside the positions (prim_nrm); then a short bench line (profile stamps check)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_pp.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 cur=$L prim=$V/libmtsgpu_pp.so prim_nrm=$V/libmtsgpu_pp2.so >> gpurun_out/r05_ab_pp.log 2>&1 || exit 1; done
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_verify.log 2>&1
