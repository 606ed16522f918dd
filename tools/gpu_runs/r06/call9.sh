#!/bin/bash
# r06 call 9: splat records of samples 2k, 2k+1 in one 32 B sector (box) and the gather
# mode's 32 B records: interleaved A/B (films compared), WRITE_SIZE per build, parity tests
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c9
mkdir -p $O
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_nopair.so
for c in C2 C3 C2g; do
  timeout -k 10 400 python -u tools/ab_variants.py $c 4 4 nopair=$B pair=$L > $O/ab_pair_$c.log 2>&1; stop $? ab_$c
done
for c in C2 C2g; do
  for v in nopair pair; do
    lib=$L; [ $v = nopair ] && lib=$B
    PROF_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/ws_${c}_$v -o pmc --output-format csv \
        -- python3 tools/prof_run.py $c 1 1 > $O/ws_${c}_$v.log 2>&1; stop $? ws_${c}_$v
  done
done
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_kernels.py \
    tests/test_gpu_parity.py tests/test_gpu_film.py tests/test_gpu_wavefront.py > $O/tests.log 2>&1; stop $? tests
echo done >> $O/status
