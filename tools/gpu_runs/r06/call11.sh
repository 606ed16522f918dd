#!/bin/bash
# r06 call 11: pair rounds (a lane renders samples 2k, 2k+1 of one pixel back to back, so
# both halves of the box record sector meet in L2) vs the plain striding (MTSG_PAIR_ROUNDS=0):
# interleaved A/B on C2 / C3 / C5 (films compared), WRITE_SIZE per arm, then the
# bench-kernel and parity tests on the new build
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c11
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_norounds.so
timeout -k 10 300 python -u tools/ab_variants.py C2 4 4 strided=$B pairs=$L > $O/ab_rounds_C2.log 2>&1; stop $? ab_C2
timeout -k 10 400 python -u tools/ab_variants.py C3 4 4 strided=$B pairs=$L > $O/ab_rounds_C3.log 2>&1; stop $? ab_C3
timeout -k 10 400 python -u tools/ab_variants.py C5 4 4 strided=$B pairs=$L > $O/ab_rounds_C5.log 2>&1; stop $? ab_C5
ws() {  # name config env...
  n=$1; c=$2; shift 2
  env "$@" timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/ws_$n -o pmc --output-format csv \
      -- python3 tools/prof_run.py $c 1 1 > $O/ws_$n.log 2>&1; stop $? ws_$n
}
ws C2_strided C2 PROF_LIB=$B
ws C2_pairs C2 PROF_LIB=$L
ws C3_pairs C3 PROF_LIB=$L
ws C5_strided C5 PROF_LIB=$B
ws C5_pairs C5 PROF_LIB=$L
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_kernels.py \
    tests/test_gpu_parity.py tests/test_gpu_film.py > $O/tests.log 2>&1; stop $? tests
echo done >> $O/status
