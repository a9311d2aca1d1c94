#!/bin/bash
# Debug build of conv_gemm.hip (LDS bound asserts; the round-2 S = 5 ring is algo 37 since round 3) linked with the other
# objects of the normal build into depth_completion_amd/debug/libdcamd.so (run on the CPU container).
set -e
cd "$(dirname "$0")/.."
python -m depth_completion_amd.build
mkdir -p depth_completion_amd/debug
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -DDC_DEBUG_LDS \
  -c depth_completion_amd/csrc/conv_gemm.hip -o depth_completion_amd/debug/conv_gemm_debug.o
objs=$(ls depth_completion_amd/build_obj/*.o | grep -v conv_gemm.hip.o)
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o depth_completion_amd/debug/libdcamd.so \
  depth_completion_amd/debug/conv_gemm_debug.o $objs
echo built depth_completion_amd/debug/libdcamd.so
