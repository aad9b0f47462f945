#!/bin/bash
# constraint_mode A/B: bench.py --constraint-mode on C2 and C5 for each build/abl variant, interleaved.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
for rep in 1 2; do
for tag in "$@"; do
  for cfg in 5 2; do
    MBIK_LIB_OVERRIDE=$PWD/build/abl/libmbik_abl_$tag.so timeout -k 10 300 python bench.py --config $cfg --constraint-mode \
      --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/r03/cm_${tag}_c${cfg}_$rep.json 2> gpurun_out/r03/cm_${tag}_c${cfg}_$rep.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'C$cfg', round(d['ms_per_step'],3), 'ms', d['config']['lanes_per_skeleton'])" gpurun_out/r03/cm_${tag}_c${cfg}_$rep.json $tag
  done
done
done
