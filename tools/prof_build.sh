#!/bin/bash
# Diagnostic build with per-phase cycle counters -> build/abl/libmbik_abl_PROF.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-result \
  -DMBIK_PROF many_bone_ik_amd/csrc/solve.hip many_bone_ik_amd/csrc/plan.cpp -o build/abl/libmbik_abl_PROF.so
