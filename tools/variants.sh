#!/bin/bash
# Timing variants of the solve library: tools/variants.sh TAG:"-DFLAG ..." ... -> build/abl/libmbik_abl_TAG.so
# (built in parallel; time them with tools/ab_run.sh / tools/variant_run.sh on the GPU box)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/abl
for spec in "$@"; do
  tag=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize -Wno-unused-result \
    $flags many_bone_ik_amd/csrc/solve.hip many_bone_ik_amd/csrc/plan.cpp -o build/abl/libmbik_abl_$tag.so 2>build/abl/$tag.log &
done
wait
ls -la build/abl/*.so
