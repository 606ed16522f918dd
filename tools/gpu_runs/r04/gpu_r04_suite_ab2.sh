#!/bin/bash
# r04: the whole GPU suite, then the wavefront profile + LDS A/B (gpu_r04_ab2.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r04_suite1.log 2>&1 || exit 1
bash tools/gpu_r04_ab2.sh
