#!/bin/bash
# r06 call 10: (a) box splat records paired per 32 B sector (film_slot) vs not, on C2 / C3;
# (b) the envmap-only set kernels without refN (MTSG_FEAT_NOREFN) vs the plain set kernels
# (MTSGPU_NO_REFN_SPEC=1, same library) on C3 / C5; films compared; WRITE_SIZE per arm;
# then the whole GPU suite on the new build
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c10
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_nopair.so
timeout -k 10 300 python -u tools/ab_variants.py C2 4 4 nopair=$B pair=$L > $O/ab_pair_C2.log 2>&1; stop $? ab_C2
for c in C3 C5; do
  timeout -k 10 400 python -u tools/ab_variants.py $c 4 4 refn=$L,MTSGPU_NO_REFN_SPEC=1 norefn=$L > $O/ab_norefn_$c.log 2>&1; stop $? ab_$c
done
ws() {  # name config env...
  n=$1; c=$2; shift 2
  env "$@" timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/ws_$n -o pmc --output-format csv \
      -- python3 tools/prof_run.py $c 1 1 > $O/ws_$n.log 2>&1; stop $? ws_$n
}
ws C2_nopair C2 PROF_LIB=$B
ws C2_pair C2 PROF_LIB=$L
ws C2g C2g PROF_LIB=$L
ws C5_refn C5 PROF_LIB=$L MTSGPU_NO_REFN_SPEC=1
ws C5_norefn C5 PROF_LIB=$L
MTSGPU_TEST_LOGDIR=$O timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests \
    > $O/gpu_suite.log 2>&1; stop $? suite
echo done >> $O/status
