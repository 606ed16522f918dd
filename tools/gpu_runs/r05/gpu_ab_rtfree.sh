#!/bin/bash
# r05: bound on C5's rough-transmittance lookup latency: every cubic2d read from one
# cache line (wrong films by design) vs the real table, megakernel and wavefront
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
L=mitsuba0.6_amd/_build/libmtsgpu.so
T=mitsuba0.6_amd/_build/variants/libmtsgpu_rtfree.so
echo "== C5 megakernel" >> gpurun_out/r05_ab_rtfree.log; timeout -k 10 300 python -u tools/ab_variants.py C5 3 4 table=$L oneline=$T >> gpurun_out/r05_ab_rtfree.log 2>&1 || exit 1
echo "== C5 wavefront" >> gpurun_out/r05_ab_rtfree.log; timeout -k 10 300 python -u tools/ab_variants.py C5 2 4 table=$L,ENGINE=wavefront oneline=$T,ENGINE=wavefront >> gpurun_out/r05_ab_rtfree.log 2>&1 || exit 1
