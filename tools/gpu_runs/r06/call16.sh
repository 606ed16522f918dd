#!/bin/bash
# r06 call 16: full-frame A/B of still longer sample runs on C3 / C5
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c16
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
timeout -k 10 400 python -u tools/ab_variants.py C3 2 1 s4=$L,MTSGPU_ROUND_SHIFT=4 s5=$L,MTSGPU_ROUND_SHIFT=5 \
    s6=$L,MTSGPU_ROUND_SHIFT=6 > $O/ab_full_C3.log 2>&1; stop $? ab_C3
timeout -k 10 500 python -u tools/ab_variants.py C5 2 1 s5=$L,MTSGPU_ROUND_SHIFT=5 s6=$L,MTSGPU_ROUND_SHIFT=6 \
    > $O/ab_full_C5.log 2>&1; stop $? ab_C5
timeout -k 10 500 python -u tools/ab_variants.py C4 2 1 s3=$L,MTSGPU_ROUND_SHIFT=3 s4=$L,MTSGPU_ROUND_SHIFT=4 \
    > $O/ab_full_C4.log 2>&1; stop $? ab_C4
echo done >> $O/status
