#!/bin/bash
# r05: the tiny-scene scan with each axis' axis-aligned planes in their own loop (numerator n_d - o_k, denominator d_k)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
B=mitsuba0.6_amd/_build/variants/libmtsgpu_base.so
T=mitsuba0.6_amd/_build/libmtsgpu.so
echo "== C2" >> gpurun_out/r05_ab_al.log; timeout -k 10 300 python -u tools/ab_variants.py C2 3 4 base=$B al=$T >> gpurun_out/r05_ab_al.log 2>&1
