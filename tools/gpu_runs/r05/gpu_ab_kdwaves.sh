#!/bin/bash
# r05: kd trace kernel at 7 and 6 waves/SIMD (72 / 80 VGPRs, fewer spills) against 8 (the build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
LOG=gpurun_out/r05_ab_kd_waves.log
for c in C4 C3; do echo "== $c" >> $LOG; AB_ENGINE=kdtree timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 w8=$L w7=$V/libmtsgpu_tw7.so w6=$V/libmtsgpu_tw6.so >> $LOG 2>&1 || exit 1; done
