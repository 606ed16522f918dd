#!/bin/bash
# The GVN scalar-PRE code-generation defect on today's source: path_kernel.hip
# (direct_kernel with its inlined any-hit traversal) built WITHOUT -mllvm -enable-pre=false,
# linked with the main build's other objects -> _build/variants/libmtsgpu_preon.so.
# On the GPU box: python tools/diag_parity.py --only=direct_shapes,indep_direct_shapes preon=<lib>
# prints the per-sample mismatch census of both libraries against the oracle.
set -eu
cd "$(dirname "$0")/../../mitsuba0.6_amd/csrc"
OUT=../_build
V=$OUT/variants/preon
mkdir -p $V
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fhip-fp32-correctly-rounded-divide-sqrt \
   -fno-gpu-flush-denormals-to-zero -mllvm -amdgpu-disable-unclustered-high-rp-reschedule -Wall -Wno-unused-function -I$OUT"
/opt/rocm/bin/hipcc $F -c path_kernel.hip -o $V/path_kernel.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/variants/libmtsgpu_preon.so $OUT/capi.o $OUT/group.o $OUT/xml_bsdf.o \
    $OUT/kdtree_build.o $OUT/scene_build.o $OUT/rtrans_host.o $V/path_kernel.o $OUT/path_f{0,1,2,3,6,7}.o $OUT/wf_kernel.o \
    $OUT/wf_shade_f{0,1,2,3,6,7}.o $OUT/film_kernel.o $OUT/probe_kernel.o
echo built $OUT/variants/libmtsgpu_preon.so
