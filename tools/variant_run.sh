#!/bin/bash
# time the default build and every build/abl/libmbik_abl_<tag>.so named on the command line
for tag in BASE "$@"; do
  if [ $tag = BASE ]; then unset MBIK_LIB_OVERRIDE; else export MBIK_LIB_OVERRIDE=$PWD/build/abl/libmbik_abl_$tag.so; fi
  echo "== $tag"; timeout -k 10 200 python tools/sweep.py 2:4096:16:4 3:65536:8:4 5:16384:32:64 2>/dev/null
done
