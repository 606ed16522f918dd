#!/bin/bash
# r06 call 29: the default bench line on the committed r06 profiles (same build): roofline fracs
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c29
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench_verify.log 2>&1
echo "bench rc=$?" >> $O/status
