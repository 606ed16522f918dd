#!/bin/bash
# r05: 5 waves/SIMD (MTSGPU_WAVES=5: BSDF-set and all-diffuse megakernels, split LDS/HBM stack) vs 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C2 C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_w5.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 w4=$L w5=$L,MTSGPU_WAVES=5 >> gpurun_out/r05_ab_w5.log 2>&1 || exit 1; done
MTSGPU_WAVES=5 timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_parity.py > gpurun_out/r05_w5_parity.log 2>&1 || exit 1
