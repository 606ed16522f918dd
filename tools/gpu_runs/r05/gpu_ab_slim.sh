#!/bin/bash
# r05: the slimmer megakernel state (wave-uniform counters, bit flags, ShFrame,
# set kernels without strictNormals) vs the round-start build; then the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_base.so
for c in C2 C3 C4 C5; do echo "== $c" >> gpurun_out/r05_ab_slim.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 base=$B cnt=mitsuba0.6_amd/_build/variants/libmtsgpu_cnt.so cntbits=mitsuba0.6_amd/_build/variants/libmtsgpu_cntbits.so slim=$L >> gpurun_out/r05_ab_slim.log 2>&1 || exit 1; done
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r05_suite_slim.log 2>&1 || exit 1
