#!/bin/bash
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
# Same-box A/B of pinned launch layouts through bench.py, interleaved twice:
#   tools/layout_ab.sh <config> <layout> [<layout> ...]     (layout = bench.py --layout)
# Prints one line per run: layout, ms per step, bitwise parity of the bench's spot check.
CFG=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
for L in "$@"; do
  timeout -k 10 150 python bench.py --config $CFG --layout $L --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lab_c${CFG}_${L//:/_}_r$rep.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/lab_c${CFG}_${L//:/_}_r$rep.json').read().strip().splitlines()[-1]);print('c$CFG', '$L', 'r$rep', round(d['ms_per_step'],4), d['parity'].get('bitwise_equal'))"
done
done
