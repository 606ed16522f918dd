#!/bin/bash
# r05: both rays of a bounce through one per-lane traversal loop (traverse_seq) at today's register pressure
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
T=mitsuba0.6_amd/_build/variants/libmtsgpu_seq.so
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_seq.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 base=$L seq=$T >> gpurun_out/r05_ab_seq.log 2>&1 || exit 1; done
