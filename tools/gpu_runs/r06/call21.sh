#!/bin/bash
# r06 call 21: tiny-scene kernels holding a pair's first splat record in registers and
# storing both as one 32 B sector (MTSG_HOLD_PAIR) against the final build: C2 A/B
# (films compared), WRITE_SIZE of both
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c21
mkdir -p $O
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_hold.so
timeout -k 10 300 python -u tools/ab_variants.py C2 4 1 base=$L hold=$B > $O/ab_hold_C2.log 2>&1; stop $? ab_C2
timeout -k 10 300 python -u tools/ab_variants.py C1 4 1 base=$L hold=$B > $O/ab_hold_C1.log 2>&1; stop $? ab_C1
for v in base hold; do
  lib=$L; [ $v = hold ] && lib=$B
  PROF_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/ws_C2_$v -o pmc --output-format csv \
      -- python3 tools/prof_run.py C2 1 1 > $O/ws_C2_$v.log 2>&1; stop $? ws_$v
done
echo done >> $O/status
