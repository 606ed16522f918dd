#!/bin/bash
# A/B builds of path_kernel.hip with extra compiler flags, linked with the main
# build's other objects:  tools/flag_variants.sh name "flags" [name "flags" ...]
#   -> _build/variants/libmtsgpu_<name>.so   (make in csrc first)
set -eu
cd "$(dirname "$0")/../mitsuba0.6_amd/csrc"
OUT=../_build
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
   -fno-gpu-flush-denormals-to-zero -I$OUT"
mkdir -p $OUT/variants/flags
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  (/opt/rocm/bin/hipcc $F $flags -Rpass-analysis=kernel-resource-usage -c path_kernel.hip \
       -o $OUT/variants/flags/pk_$name.o 2> $OUT/variants/flags/resource_$name.txt &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/variants/libmtsgpu_$name.so $OUT/capi.o $OUT/group.o \
       $OUT/kdtree_build.o $OUT/scene_build.o $OUT/rtrans_host.o $OUT/variants/flags/pk_$name.o $OUT/film_kernel.o \
       $OUT/probe_kernel.o && echo "$name ok") &
done
wait
