#!/bin/bash
# r06 call 5: packed scan (MTSG_SCAN_PK): div2 bit-check, interleaved A/B against the
# unpacked build (films compared), then the scan / bench-kernel parity tests
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c5}
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
timeout -k 10 120 mitsuba0.6_amd/_build/div2_check 67108864 > $O/div2_check.log 2>&1; stop $? div2
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_nopk.so
timeout -k 10 400 python -u tools/ab_variants.py C2 4 4 nopk=$B pk2=$L pk1=mitsuba0.6_amd/_build/variants/libmtsgpu_pk1.so > $O/ab_pk_C2.log 2>&1; stop $? ab
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_scan.py \
    tests/test_gpu_bench_kernels.py tests/test_gpu_parity.py -k "scan or bench_kernel or cornell or tile or row" > $O/tests.log 2>&1; stop $? tests
echo done >> $O/status
