#!/bin/bash
# Counter evidence for the bench layouts in one gpurun call (each rocprofv3 pass its own run and
# time limit; the first failure ends the script):
#   FETCH_SIZE and WRITE_SIZE passes per config  -> tools/traffic_from_pmc.py -> profiles/traffic.json
#   tools/valu_mix.sh's three SQ passes          -> tools/mix_entry.py      -> profiles/valu_mix.json
#   tools/replay_count.sh for C2 (the solving wave alone; needs build/abl/libmbik_replay.so)
#                                                -> tools/solver_issue.py   -> profiles/valu_mix.json
#   TAG=r04e CFGS="2 3 4 5" bash tools/r04_evidence.sh
set -o pipefail
cd "$(dirname "$0")/.."
ROOT=$PWD
TAG=${TAG:-r04e}
declare -A LAY=([2]="4:16:1:1:0:1:1" [3]="4:16:4:4:1:2:0" [4]="4:16:1:4:2:2:0" [5]="8:8:1:4:2:2:0")
echo "start $(date +%T)"
for c in ${CFGS:-2 3 4 5}; do
  OUT=$ROOT/gpurun_out/$TAG/c$c
  mkdir -p $OUT
  for ctr in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && TMPDIR=/tmp timeout -s KILL 240 rocprofv3 --pmc $ctr -d $OUT/$ctr -o run --output-format csv -- \
      python3 $ROOT/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-parity --layout ${LAY[$c]} \
      > $OUT/$ctr.json 2> $OUT/$ctr.log) || { echo "c$c $ctr pass failed"; tail -5 $OUT/$ctr.log; exit 1; }
  done
  bash tools/valu_mix.sh $TAG/mix_c$c $c ${LAY[$c]} > $OUT/mix.log 2>&1 || { echo "c$c mix passes failed"; tail -5 $OUT/mix.log; exit 1; }
  echo "c$c done $(date +%T)"
done
if [ -z "$NO_REPLAY" ]; then
  bash tools/replay_count.sh $TAG/replay 2:4096 > gpurun_out/$TAG/replay.log 2>&1 || { echo "replay failed"; tail -5 gpurun_out/$TAG/replay.log; exit 1; }
  head -2 gpurun_out/$TAG/replay.log
fi
echo "done $(date +%T)"
