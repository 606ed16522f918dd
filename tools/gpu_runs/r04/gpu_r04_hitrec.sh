#!/bin/bash
# r04: wavefront tests (hit records formed in the trace kernel), then A/B:
# megakernel, wavefront, wavefront with MTSGPU_WF_HITREC=1 (C3-C5)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_wavefront.py tests/test_gpu_kdtree.py > gpurun_out/r04_hitrec_tests.log 2>&1 || exit 1
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C3 C4 C5; do echo "== $c" >> gpurun_out/r04_ab_hitrec.log; timeout -k 10 240 python -u tools/ab_variants.py $c 3 4 mega=$L,ENGINE=megakernel wave=$L,ENGINE=wavefront,MTSGPU_WF_HITREC=0 wave_hr=$L,ENGINE=wavefront,MTSGPU_WF_HITREC=1 >> gpurun_out/r04_ab_hitrec.log 2>&1 || exit 1; done
