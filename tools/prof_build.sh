#!/bin/bash
# Diagnostic builds with the product's flags (many_bone_ik_amd/build.py FLAGS) plus one define:
#   tools/prof_build.sh            -> build/abl/libmbik_abl_PROF.so  (-DMBIK_PROF: per-phase cycle counters)
#   tools/prof_build.sh REPLAY     -> build/abl/libmbik_replay.so    (-DMBIK_REPLAY: solving wave alone, tools/replay_count.sh)
# OUT=<path> overrides the output (build/abl/ is not pushed to GPU boxes: .gpurunignore; use build/diag/)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/abl
if [ "$1" = "REPLAY" ]; then DEF=-DMBIK_REPLAY; OUT=${OUT:-build/abl/libmbik_replay.so}; else DEF=-DMBIK_PROF; OUT=${OUT:-build/abl/libmbik_abl_PROF.so}; fi
mkdir -p "$(dirname "$OUT")"
python3 -m many_bone_ik_amd.build --variant $OUT $DEF
