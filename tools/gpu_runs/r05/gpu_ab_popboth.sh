#!/bin/bash
# r05: the traversal pop reading the entry's node and distance together (MTSG_POP_BOTH)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_popboth.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 cur=$L popboth=$V/libmtsgpu_pb.so >> gpurun_out/r05_ab_popboth.log 2>&1 || exit 1; done
