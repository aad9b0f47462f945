#!/bin/bash
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
# A/B: bench C3/C4/C5 per variant (autotuned), interleaved twice
mkdir -p gpurun_out
for rep in 1 2; do
for tag in "$@"; do
 for c in ${CFGS:-3 4 5}; do
  MBIK_LIB_OVERRIDE=$PWD/build/abl/libmbik_abl_$tag.so timeout -k 10 150 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/ab_${tag}_c${c}_r$rep.json 2>gpurun_out/ab_${tag}_c${c}_r$rep.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_${tag}_c${c}_r$rep.json').read().strip().splitlines()[-1]);print('$tag c$c r$rep', round(d['ms_per_step'],3), d['config'].get('layout'))"
 done
done
done
