#!/bin/bash
# time the default build and every build/abl/libmbik_abl_<tag>.so named on the command line
CASES=${CASES:-"2:4096:4 3:65536:4 4:32768:8 5:16384:16"}
for tag in BASE "$@"; do
  if [ $tag = BASE ]; then unset MBIK_LIB_OVERRIDE; else export MBIK_LIB_OVERRIDE=$PWD/build/abl/libmbik_abl_$tag.so; fi
  echo "== $tag"; timeout -k 10 200 python tools/sweep.py $CASES 2>/dev/null
done
