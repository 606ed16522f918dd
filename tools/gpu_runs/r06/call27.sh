#!/bin/bash
# r06 call 27: BVH build knobs under sample runs (MTSGPU_LEAF_MAX, MTSGPU_SAH_CI; one library,
# the scene built per variant), full frame, C4 / C3 / C5
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c27
mkdir -p $O
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C4 C3 C5; do
  timeout -k 10 500 python -u tools/ab_variants.py $c 2 1 base=$L leaf4=$L,MTSGPU_LEAF_MAX=4 leaf12=$L,MTSGPU_LEAF_MAX=12 \
      ci05=$L,MTSGPU_SAH_CI=0.5 ci2=$L,MTSGPU_SAH_CI=2 > $O/ab_bvh_$c.log 2>&1; stop $? ab_$c
done
echo done >> $O/status
