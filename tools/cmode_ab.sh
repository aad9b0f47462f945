#!/bin/bash
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
# constraint_mode A/B: bench.py --constraint-mode on the given configs for each library, interleaved
# twice (same box), each line with its 64-skeleton bitwise parity check:
#   OUT=gpurun_out/<dir> CFGS="5 2" tools/cmode_ab.sh <lib> [...]     (<lib>: "new" = the in-tree build, or a .so path)
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/cmode_ab}
mkdir -p $OUT
for rep in 1 2; do
for lib in "$@"; do
  for cfg in ${CFGS:-5 2}; do
    tag=$(basename $lib .so)
    if [ "$lib" = new ]; then unset MBIK_LIB_OVERRIDE; else export MBIK_LIB_OVERRIDE=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --config $cfg --constraint-mode \
      --steps 10 --warmup 3 --no-cpu-baseline > $OUT/${tag}_c${cfg}_$rep.json 2> $OUT/${tag}_c${cfg}_$rep.err || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'C$cfg', 'r$rep', round(d['ms_per_step'],3), 'ms', d['config']['lanes_per_skeleton'], d['config']['skeletons_per_block'], 'rw', d['config']['layout'].get('wave_roles'), d['parity'].get('bitwise_equal'))" $OUT/${tag}_c${cfg}_$rep.json $tag
  done
done
done
unset MBIK_LIB_OVERRIDE
