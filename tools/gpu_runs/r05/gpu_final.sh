#!/bin/bash
# r05: GPU suite + smoke on the in-tree build, then its profiles (tools/prof_round.sh) and the default bench line.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
TAG=${1:-r05d}
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > gpurun_out/${TAG}_lib.sha256
timeout -k 10 700 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests \
    > gpurun_out/${TAG}_gpu_suite.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
    > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
bash tools/prof_round.sh gpurun_out/prof_${TAG} > gpurun_out/prof_${TAG}.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1 || exit 1
