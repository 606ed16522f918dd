#!/bin/bash
# r05: kd traversal with the tree's top levels read from LDS (MTSG_KD_TOP = 1024 / 1536 nodes) against the build
# (no LDS nodes); then the kd parity tests on the 1024 variant (copied over the box's scratch library)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
LOG=gpurun_out/r05_ab_kd_top.log
for c in C4 C3; do echo "== $c" >> $LOG; AB_ENGINE=kdtree timeout -k 10 400 python -u tools/ab_variants.py $c 3 16 head=$L top1024=$V/libmtsgpu_kdtop1024.so top1536=$V/libmtsgpu_kdtop1536.so >> $LOG 2>&1 || exit 1; done
cp $V/libmtsgpu_kdtop1024.so $L
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kdtree.py > gpurun_out/r05_kd_top_tests.log 2>&1
