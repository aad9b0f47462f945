#!/bin/bash
# Time build/abl/libmbik_abl_<tag>.so variants on C2/C3/C5 (tools/sweep.py), interleaved twice.
for rep in 1 2; do
for tag in "$@"; do
  export MBIK_LIB_OVERRIDE=$PWD/build/abl/libmbik_abl_$tag.so
  echo "== $tag"; timeout -k 10 200 python tools/sweep.py ${CASES:-2:4096:4 3:65536:4} 2>/dev/null || exit 1
done
done
