#!/bin/bash
# r06 call 14: longer sample runs (MTSGPU_ROUND_SHIFT 3 .. 6) on the large scenes, and
# 0 .. 3 on the gaussian C2g (gather mode: no record pairing)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c14
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C5 C3 C4; do
  timeout -k 10 400 python -u tools/ab_variants.py $c 4 4 s3=$L,MTSGPU_ROUND_SHIFT=3 s4=$L,MTSGPU_ROUND_SHIFT=4 \
      s5=$L,MTSGPU_ROUND_SHIFT=5 s6=$L,MTSGPU_ROUND_SHIFT=6 > $O/ab_shift_$c.log 2>&1; stop $? ab_$c
done
timeout -k 10 300 python -u tools/ab_variants.py C2g 4 4 s0=$L,MTSGPU_ROUND_SHIFT=0 s1=$L,MTSGPU_ROUND_SHIFT=1 \
    s2=$L,MTSGPU_ROUND_SHIFT=2 s3=$L,MTSGPU_ROUND_SHIFT=3 > $O/ab_shift_C2g.log 2>&1; stop $? ab_C2g
echo done >> $O/status
