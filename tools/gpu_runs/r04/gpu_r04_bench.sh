#!/bin/bash
# r04: smoke, the default bench line (C2 + secondary C3), and the same command
# under rocprofv3 --kernel-trace --stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${TAG:-r04_final}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_bench_prof.log 2>&1 || exit 1
