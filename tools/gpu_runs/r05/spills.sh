#!/bin/bash
# register / spill / scratch counts of the four benchmark megakernels for the
# current sources (or with extra flags: tools/gpu_runs/r05/spills.sh -DFOO=1)
cd "$(dirname "$0")/../../../mitsuba0.6_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-gpu-flush-denormals-to-zero -mllvm -amdgpu-disable-unclustered-high-rp-reschedule -mllvm -enable-pre=false \
  -Wno-unused-function -Wno-unused-variable -I../_build "$@" --cuda-device-only -c -Rpass-analysis=kernel-resource-usage \
  ../../tools/gpu_runs/r05/spill_probe.hip -o /tmp/spill_probe.o 2>&1 | grep -E "Function Name|VGPRs:|ScratchSize|Spill" | \
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' | paste - - - - - | sed -e 's/Function Name: _Z11path_kernelIL//' -e 's/EEv10MtsgLaunch//'
