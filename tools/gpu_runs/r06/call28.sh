#!/bin/bash
# r06 call 28: the round's profiles of every bench config again, the 1/4-row SQ and stall
# passes now at the full frame's sample-run length (PROF_FULL_RUNS), same build
cd $GRAFT_REPO_ROOT
CONFIGS="C2 C2g C3 C4 C5" bash tools/gpu_runs/r06/prof.sh r06c28p
