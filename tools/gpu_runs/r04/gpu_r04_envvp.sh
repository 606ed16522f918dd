#!/bin/bash
# r04: a miss's envmap value and pdf from one texel set in one call (envvp), and
# additionally roughplastic sample()'s pdf and eval in one call (rps) -- A/B on C3, C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
V=mitsuba0.6_amd/_build/variants
for c in C3 C5; do echo "== $c" >> gpurun_out/r04_ab_envvp.log; timeout -k 10 400 python -u tools/ab_variants.py $c 4 4 base=$V/libmtsgpu_base.so envvp=$V/libmtsgpu_envvp.so rps=$V/libmtsgpu_rps.so >> gpurun_out/r04_ab_envvp.log 2>&1 || exit 1; done
