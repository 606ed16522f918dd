#!/bin/bash
# r05: kd engine, TriAccel records in leaf-list order (no indices[e] -> record load chain) against the LDS-mailbox build; then the kd and scan parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3; do echo "== $c" >> gpurun_out/r05_ab_kdleaf.log; AB_ENGINE=kdtree timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 kdmb=$V/libmtsgpu_kdmb.so leaf=$L >> gpurun_out/r05_ab_kdleaf.log 2>&1 || exit 1; done
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kdtree.py tests/test_gpu_scan.py tests/test_gpu_tie_divergence.py > gpurun_out/r05_kd_scan_tests.log 2>&1
