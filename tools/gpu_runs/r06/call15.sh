#!/bin/bash
# r06 call 15: neighbour splats summed in double (order-independent spill film); full-frame
# A/B of the sample-run length on C3 / C4 / C5 (the 1/4-row A/B of calls 12 and 14 has a
# quarter of the samples per lane, so long runs leave a tail there); C3's films across shifts
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c15
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
timeout -k 10 300 python -u tools/diag_rounds.py C3 4 0 2 5 6 > $O/diag_C3.log 2>&1; stop $? diag_C3
timeout -k 10 400 python -u tools/ab_variants.py C3 3 1 s2=$L,MTSGPU_ROUND_SHIFT=2 s3=$L,MTSGPU_ROUND_SHIFT=3 \
    s4=$L,MTSGPU_ROUND_SHIFT=4 > $O/ab_full_C3.log 2>&1; stop $? ab_C3
timeout -k 10 500 python -u tools/ab_variants.py C5 3 1 s3=$L,MTSGPU_ROUND_SHIFT=3 s4=$L,MTSGPU_ROUND_SHIFT=4 \
    s5=$L,MTSGPU_ROUND_SHIFT=5 > $O/ab_full_C5.log 2>&1; stop $? ab_C5
timeout -k 10 500 python -u tools/ab_variants.py C4 3 1 s1=$L,MTSGPU_ROUND_SHIFT=1 s2=$L,MTSGPU_ROUND_SHIFT=2 \
    s3=$L,MTSGPU_ROUND_SHIFT=3 > $O/ab_full_C4.log 2>&1; stop $? ab_C4
timeout -k 10 300 python -u tools/ab_variants.py C2 3 1 s0=$L,MTSGPU_ROUND_SHIFT=0 s1=$L,MTSGPU_ROUND_SHIFT=1 \
    s2=$L,MTSGPU_ROUND_SHIFT=2 > $O/ab_full_C2.log 2>&1; stop $? ab_C2
echo done >> $O/status
