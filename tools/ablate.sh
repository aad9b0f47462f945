#!/bin/bash
# Timing-only ablation builds (results are wrong on purpose): $OUTDIR/libmbik_abl_<tag>.so
# (OUTDIR default build/abl, which is not pushed to GPU boxes -- use build/diag for a GPU run),
# each compiled with -DMBIK_ABLATE=<the tag's bits> (gd_math.h: ABL_*; the shipped mask is 0;
# MEM = every load-site ablation at once).
set -e
cd "$(dirname "$0")/.."
declare -A BIT=([SQRT]=1 [ORTHO]=2 [MATMUL]=4 [SOA]=8 [SOALDS]=16 [CONVERT]=32 [SLERP]=64 [SWING]=128 [TWIST]=256 [XCD]=512
                [WALK]=1024 [GCK]=2048 [TGT]=4096 [LOCAL]=8192 [MEM]=$((8 + 1024 + 2048 + 4096 + 8192)) [BASE]=0)
OUTDIR=${OUTDIR:-build/abl}
mkdir -p $OUTDIR
for tag in ${@:-CONVERT SLERP SWING TWIST}; do
  [ -n "${BIT[$tag]}" ] || { echo "unknown ablation $tag" >&2; exit 2; }
  python3 -m many_bone_ik_amd.build --variant $OUTDIR/libmbik_abl_$tag.so -DMBIK_ABLATE=${BIT[$tag]} >/dev/null
done
