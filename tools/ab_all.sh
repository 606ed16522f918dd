#!/bin/bash
# A/B every bench config over the given variants (tools/ab_variants.py), one step per config.
# usage: tools/ab_all.sh <out.log> name=path ...
OUT=$1; shift
mkdir -p $(dirname $OUT)
for cfg in ${CONFIGS:-C2 C3 C4 C5}; do
  echo "== $cfg" >> $OUT
  timeout -k 10 240 python3 tools/ab_variants.py $cfg ${ROUNDS:-3} ${STRIDE:-4} "$@" >> $OUT 2>&1 || { echo "step $cfg failed rc=$?" >> $OUT; exit 1; }
done
