#!/bin/bash
# r05: GPU suite on the current build, then GVN-PRE off (whole library) vs on, megakernel C2-C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r05_suite0.log 2>&1 || exit 1
L=mitsuba0.6_amd/_build/libmtsgpu.so
O=mitsuba0.6_amd/_build/variants/libmtsgpu_nopre.so
for c in C2 C3 C4 C5; do echo "== $c" >> gpurun_out/r05_ab_pre.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 pre_on=$L pre_off=$O >> gpurun_out/r05_ab_pre.log 2>&1 || exit 1; done
