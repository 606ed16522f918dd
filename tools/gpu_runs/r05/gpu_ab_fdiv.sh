#!/bin/bash
# r05: the aligned scan groups' quotients through div_by_rcp (a * RN(1/b) + two FMA corrections); then the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_base.so
echo "== C2" >> gpurun_out/r05_ab_fdiv.log; timeout -k 10 300 python -u tools/ab_variants.py C2 3 4 base=$B fdiv=$L >> gpurun_out/r05_ab_fdiv.log 2>&1 || exit 1
timeout -k 10 800 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r05_gpu_suite_fdiv.log 2>&1
