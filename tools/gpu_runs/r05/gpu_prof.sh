#!/bin/bash
# r05: profiles of the current build (tools/prof_round.sh), then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
OUT=gpurun_out/prof_${1:-r05}
bash tools/prof_round.sh $OUT > gpurun_out/prof_${1:-r05}.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${1:-r05}.log 2>&1 || exit 1
