#!/bin/bash
# r06 call 20: the sample-run parity test and the bench-kernel tests against the committed
# r06 profiles, on the final build
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c20
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_sample_runs.py \
    tests/test_gpu_bench_kernels.py tests/test_spill_order.py > $O/tests.log 2>&1
echo "tests rc=$?" >> $O/status
