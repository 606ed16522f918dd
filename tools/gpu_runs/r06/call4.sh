#!/bin/bash
# r06 call 4: C4's diverging ray through every GPU traversal
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c4
mkdir -p $O
timeout -k 10 300 python -u tools/diag_c4_ray.py > $O/diag_c4_ray.log 2>&1; echo "diag rc=$?" >> $O/status
