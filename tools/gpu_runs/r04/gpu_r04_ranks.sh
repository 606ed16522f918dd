#!/bin/bash
# r04: bench.py's N-rank path with the ranks sharing the box's GPU, then one
# cache pass (L2 hit rate, L1 -> L2 requests) over C3 / C4 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_bench_ranks.py > gpurun_out/r04_ranks_tests.log 2>&1 || exit 1
for cfg in C3 C4 C5; do
  timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace \
      -d gpurun_out/r04cache/pmc_${cfg} -o pmc --output-format csv -- python3 tools/prof_run.py $cfg 1 4 > gpurun_out/r04cache/pmc_${cfg}.log 2>&1 || exit 1
done
