#!/bin/bash
# r04: parity of the rebuilt engines, then an interleaved A/B on C2-C5:
# megakernel before / after launch_fresh, and the one-item-per-thread wavefront
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wavefront.py tests/test_gpu_kdtree.py tests/test_gpu_parity.py > gpurun_out/r04_ab1_tests.log 2>&1 || exit 1
L=mitsuba0.6_amd/_build/libmtsgpu.so
O=mitsuba0.6_amd/_build/variants/libmtsgpu_nofresh.so
for c in C2 C3 C4 C5; do echo "== $c" >> gpurun_out/r04_ab1.log; timeout -k 10 240 python -u tools/ab_variants.py $c 3 4 mega_old=$O,ENGINE=megakernel mega_new=$L,ENGINE=megakernel wave_new=$L,ENGINE=wavefront >> gpurun_out/r04_ab1.log 2>&1 || exit 1; done
