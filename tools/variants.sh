#!/bin/bash
# Timing variants of the solve library: tools/variants.sh TAG:"-DFLAG ..." ... -> build/abl/libmbik_abl_TAG.so
# (each build's translation units compile in parallel; time them with tools/ab_run.sh / tools/variant_run.sh on the GPU box)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/abl
for spec in "$@"; do
  tag=${spec%%:*}; flags=${spec#*:}
  python3 -m many_bone_ik_amd.build --variant build/abl/libmbik_abl_$tag.so $flags >build/abl/$tag.log 2>&1
done
ls -la build/abl/*.so
