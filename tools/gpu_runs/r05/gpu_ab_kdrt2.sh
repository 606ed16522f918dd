#!/bin/bash
# r05: kd traversal, two newest stack entries in registers (kdrt2) against one (the build); then the kd parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3; do echo "== $c" >> gpurun_out/r05_ab_kdrt2.log; AB_ENGINE=kdtree timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 regtop1=$L regtop2=$V/libmtsgpu_kdrt2.so >> gpurun_out/r05_ab_kdrt2.log 2>&1 || exit 1; done
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kdtree.py tests/test_gpu_tie_divergence.py > gpurun_out/r05_kd_tests_regtop.log 2>&1
