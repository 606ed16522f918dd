#!/bin/bash
# r05: SAH build knobs on today's traversal (leaf records read ahead since round 5): triangle-test cost and leaf size
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
LOG=gpurun_out/r05_ab_sah.log
for c in C4 C3 C5; do echo "== $c" >> $LOG; timeout -k 10 400 python -u tools/ab_variants.py $c 3 4 base=$L ci15=$L,MTSGPU_SAH_CI=1.5 ci2=$L,MTSGPU_SAH_CI=2 ci07=$L,MTSGPU_SAH_CI=0.7 leaf12ci15=$L,MTSGPU_SAH_CI=1.5,MTSGPU_LEAF_MAX=12 >> $LOG 2>&1 || exit 1; done
