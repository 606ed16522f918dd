#!/bin/bash
# r04: parity after dropping px/py/j from the path state, then A/B against the
# previous build (C2-C5, 1/4 of the rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_wavefront.py tests/test_gpu_sfmt.py > gpurun_out/r04_slim_tests.log 2>&1 || exit 1
L=mitsuba0.6_amd/_build/libmtsgpu.so
O=mitsuba0.6_amd/_build/variants/libmtsgpu_prev.so
for c in C2 C3 C4 C5; do echo "== $c" >> gpurun_out/r04_ab_slim.log; timeout -k 10 300 python -u tools/ab_variants.py $c 4 4 prev=$O,ENGINE=megakernel slim=$L,ENGINE=megakernel >> gpurun_out/r04_ab_slim.log 2>&1 || exit 1; done
