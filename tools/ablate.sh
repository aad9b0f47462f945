#!/bin/bash
# Timing-only ablation builds (results are wrong on purpose): build/abl/libmbik_abl_<tag>.so,
# each compiled with -DMBIK_ABLATE=<the tag's bit> (gd_math.h: ABL_*; the shipped mask is 0).
set -e
cd "$(dirname "$0")/.."
declare -A BIT=([SQRT]=1 [ORTHO]=2 [MATMUL]=4 [SOA]=8 [SOALDS]=16 [CONVERT]=32 [SLERP]=64 [SWING]=128 [TWIST]=256 [XCD]=512)
mkdir -p build/abl
for tag in ${@:-CONVERT SLERP SWING TWIST}; do
  [ -n "${BIT[$tag]}" ] || { echo "unknown ablation $tag" >&2; exit 2; }
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-slp-vectorize -Wno-unused-result \
    -DMBIK_ABLATE=${BIT[$tag]} many_bone_ik_amd/csrc/solve.hip many_bone_ik_amd/csrc/plan.cpp -o build/abl/libmbik_abl_$tag.so &
done
wait
