#!/bin/bash
# r06 call 3: the C4 bench-kernel mismatch diagnosed; the gather-mode film (gaussian)
# tests; the bench kernels vs the oracle; C2 / C2g timing with kernel stats.
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c3
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
timeout -k 10 300 python -u tools/diag_bench_kernel.py C4 299 6 > $O/diag_C4.log 2>&1; stop $? diag
MTSGPU_TEST_LOGDIR=$O timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread \
    tests/test_gpu_bench_kernels.py tests/test_gpu_rccl.py tests/test_gpu_parity.py tests/test_gpu_film.py \
    tests/test_gpu_wavefront.py tests/test_gpu_group.py > $O/tests.log 2>&1; stop $? tests
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bench_C2g -o bench --output-format csv \
    -- python3 bench.py --config C2g --steps 3 --warmup 1 --no-cpu-baseline --secondary C2 > $O/bench_C2g.log 2>&1; stop $? bench
echo done >> $O/status
