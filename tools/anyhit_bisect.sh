#!/bin/bash
# Diagnostics: LLVM -opt-bisect-limit builds of path_kernel.hip with the
# any-hit query inlined into direct_kernel (-DMTSG_ANYHIT_INLINE), for
# bisecting which optimisation pass run makes direct_kernel<true, 6> (the
# analytic-shape scene) answer shadow rays wrongly.
#   tools/anyhit_bisect.sh N1 N2 ...  ->  _build/variants/libmtsgpu_bis<N>.so
# The other objects come from the main build (make in csrc first).
# Result: the first wrong build is run 122502, GVN on
# direct_kernel<true, 6>; with -mllvm -enable-pre=false the -O3 build is exact.
set -eu
cd "$(dirname "$0")/../mitsuba0.6_amd/csrc"
OUT=../_build
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
   -fno-gpu-flush-denormals-to-zero -I$OUT -DMTSG_ANYHIT_INLINE"
mkdir -p $OUT/variants/bis
for n in "$@"; do
  (/opt/rocm/bin/hipcc $F -mllvm -opt-bisect-limit=$n -c path_kernel.hip -o $OUT/variants/bis/pk_$n.o 2> /dev/null &&
   /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/variants/libmtsgpu_bis$n.so $OUT/capi.o $OUT/group.o \
       $OUT/kdtree_build.o $OUT/scene_build.o $OUT/rtrans_host.o $OUT/variants/bis/pk_$n.o $OUT/film_kernel.o \
       $OUT/probe_kernel.o && echo "bis$n ok") &
done
wait
