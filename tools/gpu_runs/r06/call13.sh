#!/bin/bash
# r06 call 13: film determinism across sample-run lengths (C3 films differed between
# MTSGPU_ROUND_SHIFT 0 and >= 2 in call 12): repeated renders per shift, then the
# bench-kernel band parity test at each shift
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06c13
mkdir -p $O
sha256sum mitsuba0.6_amd/_build/libmtsgpu.so > $O/lib.sha256
stop() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc at $2" >> $O/status; exit $rc; fi; echo "$2 rc=$rc" >> $O/status; }
timeout -k 10 300 python -u tools/diag_rounds.py C3 4 0 1 2 3 > $O/diag_C3.log 2>&1; stop $? diag_C3
timeout -k 10 300 python -u tools/diag_rounds.py C5 4 0 3 4 > $O/diag_C5.log 2>&1; stop $? diag_C5
for s in 0 2 3 4; do
  MTSGPU_ROUND_SHIFT=$s timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread \
      tests/test_gpu_bench_kernels.py -k "band" > $O/band_s$s.log 2>&1; stop $? band_s$s
done
echo done >> $O/status
