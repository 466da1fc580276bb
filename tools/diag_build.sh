#!/bin/bash
# Rebuild libopenr_hip in place with diagnostic macros (GPU box scratch copy
# only; never commit the result): tools/diag_build.sh -DORH_DIAG_NO_DIST_STORE
set -e
cd "$(dirname "$0")/.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value -Wno-unused-result "$@" \
  -o openr_amd/lib/libopenr_hip.so openr_amd/csrc/orh_api.hip openr_amd/csrc/kernels/spf_kernels.hip \
  openr_amd/csrc/kernels/route_kernels.hip openr_amd/csrc/kernels/whatif_kernels.hip \
  openr_amd/csrc/kernels/ksp_kernels.hip
