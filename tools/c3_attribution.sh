#!/bin/bash
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
# where C3's waves wait (65,536 skeletons x 32 bones / 4 effectors, no
# constraints), on the shipped classic layout and on the wave-roles layout, with the round-5
# attribution tooling:
#   1. PMC classes per layout (tools/stall_counters.sh, TRAFFIC=1: FETCH_SIZE / WRITE_SIZE too);
#   2. load-site ablations (build/diag/libmbik_abl_<tag>.so from
#      OUTDIR=build/diag tools/ablate.sh WALK LOCAL SOA MEM; results wrong on purpose, time only;
#      BASE_LIB: the library they were built from, default the in-tree one);
#   3. the phase split (build/diag/libmbik_abl_PROF.so, tools/prof_phases.py).
# Every step has its own time limit and the first failure ends the script.    TAG=r06c tools/c3_attribution.sh
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-c3attr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
CLASSIC=${CLASSIC:-4:16:4:4:1:2:0:0}
ROLES=${ROLES_LAYOUT:-4:64:1:0:2:2:0:1}
echo "counters $(date +%T)"
TRAFFIC=1 timeout -k 10 600 bash tools/stall_counters.sh $TAG 3:$CLASSIC 3:$ROLES > $OUT/counters.log 2>&1 || { echo counters failed; exit 1; }
echo "ablations $(date +%T)"
TAG=$TAG STEPS=10 timeout -k 10 600 bash tools/ab_env.sh "base||${BASE_LIB:--}" "WALK||build/diag/libmbik_abl_WALK.so" \
  "LOCAL||build/diag/libmbik_abl_LOCAL.so" "SOA||build/diag/libmbik_abl_SOA.so" "MEM||build/diag/libmbik_abl_MEM.so" \
  -- 3:$CLASSIC 3:$ROLES > $OUT/ablations.log 2>&1 || { echo ablations failed; tail -5 $OUT/ablations.log; exit 1; }
cat $OUT/ablations.log
echo "phases $(date +%T)"
C=(${CLASSIC//:/ }); R=(${ROLES//:/ })
MBIK_LIB_OVERRIDE=$PWD/build/diag/libmbik_abl_PROF.so timeout -k 10 300 python tools/prof_phases.py \
  3:65536:${C[0]}:${C[1]}:${C[2]}:${C[3]}:${C[4]}:${C[5]} 3:65536:${R[0]}:${R[1]}:${R[2]}:${R[3]}:${R[4]}:${R[5]}:1 \
  > $OUT/phases.jsonl 2> $OUT/phases.err || { echo phases failed; tail -5 $OUT/phases.err; exit 1; }
cat $OUT/phases.jsonl | cut -c1-400
echo "done $(date +%T)"
