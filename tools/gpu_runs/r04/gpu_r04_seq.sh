#!/bin/bash
# r04: parity with the sequential two-ray traversal, then A/B against the
# separate traversals (C3-C5, 1/4 of the rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/r04_seq_tests.log 2>&1 || exit 1
L=mitsuba0.6_amd/_build/libmtsgpu.so
O=mitsuba0.6_amd/_build/variants/libmtsgpu_noseq.so
for c in C3 C4 C5; do echo "== $c" >> gpurun_out/r04_ab_seq.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 sep=$O,ENGINE=megakernel seq=$L,ENGINE=megakernel >> gpurun_out/r04_ab_seq.log 2>&1 || exit 1; done
