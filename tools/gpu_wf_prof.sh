#!/bin/bash
# Kernel-level profile of the wavefront engine vs the megakernel on C3-C5
# (rocprofv3 --kernel-trace --stats over tools/prof_run.py, 1/4 of the rows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${TAG:-r04_wfprof}
for c in ${CFGS:-C3 C4 C5}; do
  for e in ${ENGINES:-wavefront}; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${c}_$e -o run -- python3 -u tools/prof_run.py $c 2 4 $e > gpurun_out/${TAG}_${c}_$e.log 2>&1 || exit 1
  done
done
