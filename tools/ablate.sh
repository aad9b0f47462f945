#!/bin/bash
# Timing-only ablation builds (results are wrong on purpose): libmbik_<tag>.so
set -e
cd "$(dirname "$0")/.."
for tag in ${@:-CONVERT SLERP SWING TWIST}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-result \
    -DMBIK_ABLATE_$tag many_bone_ik_amd/csrc/solve.hip many_bone_ik_amd/csrc/plan.cpp -o build/abl/libmbik_abl_$tag.so &
done
wait
