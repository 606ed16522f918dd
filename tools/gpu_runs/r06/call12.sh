#!/bin/bash
# r06 call 12: megakernel sample-run length 2^s (MTSGPU_ROUND_SHIFT = 0 .. 4, one library):
# interleaved A/B on C2 / C3 / C4 / C5 (films compared), WRITE_SIZE at s = 2
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c12
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
L=mitsuba0.6_amd/_build/libmtsgpu.so
for c in C2 C3 C4 C5; do
  timeout -k 10 400 python -u tools/ab_variants.py $c 4 4 s0=$L,MTSGPU_ROUND_SHIFT=0 s1=$L,MTSGPU_ROUND_SHIFT=1 \
      s2=$L,MTSGPU_ROUND_SHIFT=2 s3=$L,MTSGPU_ROUND_SHIFT=3 s4=$L,MTSGPU_ROUND_SHIFT=4 > $O/ab_rounds_$c.log 2>&1; stop $? ab_$c
done
for c in C2 C3; do
  MTSGPU_ROUND_SHIFT=2 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/ws_${c}_s2 -o pmc --output-format csv \
      -- python3 tools/prof_run.py $c 1 1 > $O/ws_${c}_s2.log 2>&1; stop $? ws_$c
done
echo done >> $O/status
