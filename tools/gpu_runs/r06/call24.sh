#!/bin/bash
# r06 call 24: film_gather with two output rows per thread (MTSG_GATHER_ROWS=2, the in-tree
# build) against one (variant): C2g A/B, films compared; the gaussian parity tests
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c24
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_grows1.so
timeout -k 10 300 python -u tools/ab_variants.py C2g 4 1 rows1=$B rows2=$L > $O/ab_gather_rows_C2g.log 2>&1; stop $? ab_C2g
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_kernels.py \
    tests/test_gpu_parity.py tests/test_gpu_film.py tests/test_gpu_wavefront.py > $O/tests.log 2>&1; stop $? tests
echo done >> $O/status
