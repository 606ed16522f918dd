#!/bin/bash
# r06 call 25: the build with two-row film_gather: the whole GPU suite and
# smoke, then the round's profiles of every bench config
cd $GRAFT_REPO_ROOT
bash tools/gpu_runs/r06/suite.sh r06c25 || exit $?
grep -q "suite rc=0" gpurun_out/r06c25/status && grep -q "smoke rc=0" gpurun_out/r06c25/status || exit 1
CONFIGS="C2 C2g C3 C4 C5" bash tools/gpu_runs/r06/prof.sh r06c25p
