#!/bin/bash
# r06: the whole GPU suite and smoke on the in-tree build (TAG names the output)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06_suite}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
MTSGPU_TEST_LOGDIR=$O timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests \
    > $O/gpu_suite.log 2>&1; rc=$?; echo "suite rc=$rc" >> $O/status
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/smoke.log 2>&1
echo "smoke rc=$?" >> $O/status
