#!/bin/bash
# r05: wavefront / kd-tree engine tests after the per-region queue capacities changed
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_wavefront.py tests/test_gpu_kdtree.py > gpurun_out/r05_wf_tests.log 2>&1 || exit 1
