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
# (revisions before round 6 had one solve.hip translation unit)
if [ -f $TMP/many_bone_ik_amd/csrc/solve.hip ]; then
  /opt/rocm/bin/hipcc $FLAGS $TMP/many_bone_ik_amd/csrc/solve.hip $TMP/many_bone_ik_amd/csrc/plan.cpp -o build/abl/libmbik_abl_$TAG.so 2>/dev/null
else
  python3 -m many_bone_ik_amd.build --variant build/abl/libmbik_abl_$TAG.so --csrc $TMP/many_bone_ik_amd/csrc >/dev/null 2>&1
fi
python3 -m many_bone_ik_amd.build --variant build/abl/libmbik_abl_NEW.so >/dev/null 2>&1
rm -rf $TMP
ls -la build/abl/libmbik_abl_$TAG.so build/abl/libmbik_abl_NEW.so
