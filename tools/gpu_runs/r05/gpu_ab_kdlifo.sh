#!/bin/bash
# r05: kd engine, the Havran stack as a by-value LIFO (one stack read per pop) against HEAD; then the kd and scan parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3; do echo "== $c" >> gpurun_out/r05_ab_kdlifo.log; AB_ENGINE=kdtree timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 head=$V/libmtsgpu_kdhead.so lifo=$L >> gpurun_out/r05_ab_kdlifo.log 2>&1 || exit 1; done
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kdtree.py tests/test_gpu_scan.py tests/test_gpu_tie_divergence.py > gpurun_out/r05_kd_scan_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_kd_C4 -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_run.py C4 1 16 kdtree > $GRAFT_REPO_ROOT/gpurun_out/prof_kd_C4.log 2>&1
