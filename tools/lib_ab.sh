#!/bin/bash
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
# Same-box A/B of the in-tree library against build/abl/libmbik_abl_<tag>.so on pinned layouts,
# interleaved twice:   [ABDIR=build/diag] [ENV_NEW="K=V"] tools/lib_ab.sh <tag> <config>:<layout> [...]
# (build/abl is not pushed to GPU boxes: use ABDIR=build/diag there)
TAG=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
for CL in "$@"; do
  CFG=${CL%%:*}; L=${CL#*:}
  for lib in new $TAG; do
    if [ $lib = new ]; then unset MBIK_LIB_OVERRIDE; else export MBIK_LIB_OVERRIDE=$PWD/${ABDIR:-build/abl}/libmbik_abl_$lib.so; fi
    out=gpurun_out/libab_${lib}_c${CFG}_${L//:/_}_r$rep.json
    timeout -k 10 150 python bench.py --config $CFG --layout $L --steps 20 --warmup 3 --no-cpu-baseline > $out 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('$lib', 'c$CFG', '$L', 'r$rep', round(d['ms_per_step'],4), d['parity'].get('bitwise_equal'))"
  done
done
done
unset MBIK_LIB_OVERRIDE
