#!/bin/bash
# r04: kd-tree engine parity + the BVH-vs-kd tie divergence, then A/B of the
# kd trace kernel's LDS stack/mailbox (C3, C4; 1/16 of the rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kdtree.py tests/test_gpu_tie_divergence.py > gpurun_out/r04_kd_tests.log 2>&1 || exit 1
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C3 C4; do echo "== $c" >> gpurun_out/r04_ab_kd.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 16 kd_scratch=$L,ENGINE=kdtree,MTSGPU_KD_LDS=0 kd_lds=$L,ENGINE=kdtree mega=$L,ENGINE=megakernel >> gpurun_out/r04_ab_kd.log 2>&1 || exit 1; done
