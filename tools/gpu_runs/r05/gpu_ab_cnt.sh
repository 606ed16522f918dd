#!/bin/bash
# r05: wave-uniform counters (cnt) and bitfield path flags (cntbits) vs HEAD, megakernel C2-C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
A=mitsuba0.6_amd/_build/variants/libmtsgpu_cnt.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_cntbits.so
for c in C2 C3 C4 C5; do echo "== $c" >> gpurun_out/r05_ab_cnt.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 base=$L cnt=$A cntbits=$B >> gpurun_out/r05_ab_cnt.log 2>&1 || exit 1; done
