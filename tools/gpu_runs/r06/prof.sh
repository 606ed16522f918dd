#!/bin/bash
# r06: profiles of the in-tree build (tools/prof_round.sh) for the configs in $CONFIGS,
# optionally the write-granularity passes (WG=1) and the default bench line (BENCH=1)
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06p}
O=gpurun_out/$TAG
mkdir -p $O
if [ "${WG:-0}" = 1 ]; then
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/write_gran -o pmc --output-format csv \
      -- mitsuba0.6_amd/_build/write_gran > $O/write_gran.log 2>&1 || { echo "write_gran rc=$?" >> $O/status; exit 1; }
fi
bash tools/prof_round.sh $O/prof > $O/prof.log 2>&1 || { echo "prof rc=$?" >> $O/status; exit 1; }
echo "prof ok" >> $O/status
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench_default.log 2>&1; echo "bench rc=$?" >> $O/status
fi
