#!/bin/bash
# r05: the kd engine's trace kernel with its hashed mailbox in LDS (kdmb) and with the first 3 stack entries too (kdmb2), both at 8 waves/SIMD; and the scratch-only kernel at 4 waves (kdw4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 AB_ENGINE=kdtree
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3; do echo "== $c" >> gpurun_out/r05_ab_kdmb.log; timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 base=$L kdmb=$V/libmtsgpu_kdmb.so kdmb2=$V/libmtsgpu_kdmb2.so kdw4=$V/libmtsgpu_kdw4.so >> gpurun_out/r05_ab_kdmb.log 2>&1 || exit 1; done
