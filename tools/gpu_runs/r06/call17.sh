#!/bin/bash
# r06 call 17: the whole GPU suite, smoke and the default bench line on the build with
# adaptive sample runs and double-summed neighbour splats
cd $GRAFT_REPO_ROOT
bash tools/gpu_runs/r06/suite.sh r06c17 || exit $?
grep -q "suite rc=0" gpurun_out/r06c17/status && grep -q "smoke rc=0" gpurun_out/r06c17/status || exit 1
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r06c17/bench_default.log 2>&1
echo "bench rc=$?" >> gpurun_out/r06c17/status
