#!/bin/bash
# r05: the whole GPU suite and smoke on the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > gpurun_out/r05_final_lib.sha256
timeout -k 10 700 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests \
    > gpurun_out/r05_gpu_suite_final.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" >> gpurun_out/r05_gpu_suite_final.log 2>&1
