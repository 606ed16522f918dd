#!/bin/bash
# r06 call 19: TriAccel records as non-temporal loads (MTSG_TRI_NT=1) against the final
# build, full frame, C4 / C3 / C5 (films compared)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c19
mkdir -p $O
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
B=mitsuba0.6_amd/_build/variants/libmtsgpu_trint.so
for c in C4 C3 C5; do
  timeout -k 10 500 python -u tools/ab_variants.py $c 3 1 base=$L trint=$B > $O/ab_trint_$c.log 2>&1; stop $? ab_$c
done
echo done >> $O/status
