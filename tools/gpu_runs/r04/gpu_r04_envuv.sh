#!/bin/bash
# r04: the envmap's (u, v) formed once per miss for both evalEnvironment and
# internalPdfDirection -- A/B against the previous build on C3 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
B=mitsuba0.6_amd/_build/variants/libmtsgpu_base.so
N=mitsuba0.6_amd/_build/variants/libmtsgpu_envuv.so
for c in C3 C5; do echo "== $c" >> gpurun_out/r04_ab_envuv.log; timeout -k 10 300 python -u tools/ab_variants.py $c 4 4 base=$B envuv=$N >> gpurun_out/r04_ab_envuv.log 2>&1 || exit 1; done
