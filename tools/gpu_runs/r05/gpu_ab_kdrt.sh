#!/bin/bash
# r05: kd traversal with the newest stack entry held in registers (MTSG_KD_REGTOP)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3; do echo "== $c" >> gpurun_out/r05_ab_kdrt.log; AB_ENGINE=kdtree timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 cur=$L regtop=$V/libmtsgpu_kdrt.so >> gpurun_out/r05_ab_kdrt.log 2>&1 || exit 1; done
