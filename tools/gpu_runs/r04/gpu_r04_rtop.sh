#!/bin/bash
# r04: A/B of the register-cached traversal stack top (MTSG_REG_TOP), C2-C5,
# then the parity tests on that build
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants/libmtsgpu_rtop.so
for c in C2 C3 C4 C5; do echo "== $c" >> gpurun_out/r04_ab_rtop.log; timeout -k 10 300 python -u tools/ab_variants.py $c 4 4 base=$L,ENGINE=megakernel rtop=$V,ENGINE=megakernel >> gpurun_out/r04_ab_rtop.log 2>&1 || exit 1; done
