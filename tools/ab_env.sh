#!/bin/bash
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
# Same-box A/B of library variants on pinned layouts, interleaved REPS times (default 2):
#   tools/ab_env.sh "<label>|<env assignments>|<lib .so or ->" ... -- <config>:<layout> [...]
# e.g.  tools/ab_env.sh "rec|MBIK_RW_REC=1|-" "norec|MBIK_RW_REC=0|-" "base||build/diag/libmbik_abl_BASE.so" \
#         -- 4:4:64:1:0:2:2:0:1 5:8:64:2:0:2:2:0:1
# Each line: label, config, layout, rep, ms per step, bitwise parity of the bench's checked skeletons.
# Output JSON lines under gpurun_out/${TAG:-ab}/.
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
shift
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for rep in $(seq 1 ${REPS:-2}); do
for CL in "$@"; do
  CFG=${CL%%:*}; L=${CL#*:}
  for v in "${VARS[@]}"; do
    IFS='|' read -r label envs lib <<< "$v"
    out=$OUT/${label}_c${CFG}_${L//:/_}_r$rep.json
    ( [ "$lib" != "-" ] && [ -n "$lib" ] && export MBIK_LIB_OVERRIDE=$PWD/$lib
      for e in ${envs//,/ }; do export "$e"; done
      exec timeout -k 10 ${AB_TIMEOUT:-200} python bench.py --config $CFG --layout $L --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
        ${EXTRA} > $out 2>$out.err ) || { echo "FAILED $label c$CFG"; tail -3 $out.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$out').read().strip().splitlines()[-1]);print('$label', 'c$CFG', '$L', 'r$rep', round(d['ms_per_step'],4), (d.get('parity') or {}).get('bitwise_equal'))"
  done
done
done
