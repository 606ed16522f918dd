#!/bin/bash
# r05: pop with both LDS reads issued before one wait (MTSG_POP_ONE_WAIT) against the node read first
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
V=mitsuba0.6_amd/_build/variants
for c in C4 C3 C5; do echo "== $c" >> gpurun_out/r05_ab_pop_onewait.log; timeout -k 10 300 python -u tools/ab_variants.py $c 3 4 popboth=$L onewait=$V/libmtsgpu_p1.so >> gpurun_out/r05_ab_pop_onewait.log 2>&1 || exit 1; done
