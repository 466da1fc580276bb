#!/bin/bash
# Build an experiment variant of libopenr_hip.so with extra defines into
# build_var/NAME/ (not gpurun-ignored: variants travel with the snapshot and
# are selected on the box with LD_LIBRARY_PATH=build_var/NAME).
#   tools/build_variant.sh NAME -DFLAG[=V] ...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build_var/$NAME"
SRCS=$(python3 -c "import sys; sys.path.insert(0, '$ROOT'); from openr_amd import build; print(' '.join(build.HIP_SRCS))")
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value -Wno-unused-result \
  "$@" -o "$ROOT/build_var/$NAME/libopenr_hip.so" $SRCS
echo "built build_var/$NAME/libopenr_hip.so $*"
