#!/bin/bash
# GPU check of the wavefront engine: its parity tests, then an interleaved
# megakernel / wavefront A/B on C3-C5 (tools/ab_variants.py, 1/4 of the rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 420 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wavefront.py tests/test_gpu_kdtree.py > gpurun_out/r04_wf1_tests.log 2>&1 && \
L=mitsuba0.6_amd/_build/libmtsgpu.so && \
for c in C3 C4 C5; do echo "== $c" >> gpurun_out/r04_wf1_ab.log; timeout -k 10 200 python -u tools/ab_variants.py $c 3 4 mega=$L,ENGINE=megakernel wave=$L,ENGINE=wavefront >> gpurun_out/r04_wf1_ab.log 2>&1 || exit 1; done
