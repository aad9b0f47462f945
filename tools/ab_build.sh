#!/bin/bash
# A/B builds for tools/variant_check.py: build/abl/libmbik_abl_<TAG>.so from the csrc of a git
# revision (default HEAD), and build/abl/libmbik_abl_NEW.so from the working tree, both with the
# product flags.   tools/ab_build.sh [REV [TAG]]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; TAG=${2:-BASE}
FLAGS=$(python3 -c "from many_bone_ik_amd.build import FLAGS; print(' '.join(FLAGS))")
TMP=$(mktemp -d)
git archive $REV many_bone_ik_amd/csrc include | tar -x -C $TMP
mkdir -p build/abl
/opt/rocm/bin/hipcc $FLAGS $TMP/many_bone_ik_amd/csrc/solve.hip $TMP/many_bone_ik_amd/csrc/plan.cpp -o build/abl/libmbik_abl_$TAG.so 2>/dev/null &
/opt/rocm/bin/hipcc $FLAGS many_bone_ik_amd/csrc/solve.hip many_bone_ik_amd/csrc/plan.cpp -o build/abl/libmbik_abl_NEW.so 2>/dev/null &
wait
rm -rf $TMP
ls -la build/abl/libmbik_abl_$TAG.so build/abl/libmbik_abl_NEW.so
