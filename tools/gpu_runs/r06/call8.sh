#!/bin/bash
# r06 call 8: film_gather with the value channels in packed pairs: interleaved A/B on C2g
# (films compared) and the gather parity tests
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c8
mkdir -p $O
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_gnopk.so
timeout -k 10 400 python -u tools/ab_variants.py C2g 5 4 gnopk=$B gpk=$L > $O/ab_gather_pk.log 2>&1; stop $? ab
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks -o ks --output-format csv -- python3 tools/ab_variants.py C2g 2 4 gnopk=$B gpk=$L > $O/ks.log 2>&1; stop $? ks
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_kernels.py \
    tests/test_gpu_parity.py tests/test_gpu_film.py tests/test_gpu_wavefront.py -k "C2g or gaussian or develop_rendered" > $O/tests.log 2>&1; stop $? tests
echo done >> $O/status
