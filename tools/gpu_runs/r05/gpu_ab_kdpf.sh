#!/bin/bash
# r05: kd leaf loop reading the next record ahead (kdpf) against the current build; then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3; do echo "== $c" >> gpurun_out/r05_ab_kdpf.log; AB_ENGINE=kdtree timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 cur=$L kdpf=$V/libmtsgpu_kdpf.so >> gpurun_out/r05_ab_kdpf.log 2>&1 || exit 1; done
timeout -k 10 1200 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r05_gpu_suite.log 2>&1
