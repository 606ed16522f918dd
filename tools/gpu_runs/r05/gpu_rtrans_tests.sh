#!/bin/bash
# r05: C5 on the reference's ggx.dat layers (tests/golden/rtrans_c5_ggx_layers.npz), then a bench line on the stamped profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py::test_c5_reference_table_layers_bitexact tests/test_gpu_fullsize.py::test_c5_row_band_on_reference_table_layers \
    > gpurun_out/r05_rtrans_ref_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r05d_bench_verify.log 2>&1 || exit 1
