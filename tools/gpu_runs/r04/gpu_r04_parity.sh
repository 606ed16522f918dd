#!/bin/bash
# r04: parity tests after the any-hit / GVN-PRE change and the ANA set-kernel crosscheck
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py > gpurun_out/r04_parity2.log 2>&1
