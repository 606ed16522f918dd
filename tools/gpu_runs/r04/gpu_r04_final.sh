#!/bin/bash
# r04 final: the whole GPU suite, the round profiles (stamped), smoke + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04f_suite.log 2>&1 || exit 1
bash tools/prof_round.sh gpurun_out/r04fprof || exit 1
TAG=r04f bash tools/gpu_r04_bench.sh
