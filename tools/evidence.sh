#!/bin/bash
# GPU evidence passes, one gpurun call each (every step under its own time limit; the first step
# that ends badly ends the script).  Subcommands:
#
#   tools/evidence.sh call               TAG, TESTS (default: the whole -m gpu suite), SMOKE=1, BENCH="args;args"
#       the -m gpu tests, then optionally smoke() and bench lines          -> gpurun_out/$TAG/
#   tools/evidence.sh final              TAG
#       the whole suite, smoke(), the default bench line (C2) with its rocprofv3 kernel stats,
#       the autotuned C3 / C4 / C5 lines and the constraint_mode C5 / C2 lines -> gpurun_out/$TAG/
#   tools/evidence.sh counters           TAG, CFGS="2 3 4 5", LAYOUTS="c:layout ..." (default: the bench's picks)
#       FETCH_SIZE / WRITE_SIZE passes (tools/traffic_from_pmc.py -> profiles/traffic.json) and the
#       VALU mix (tools/valu_mix.sh -> tools/mix_entry.py -> profiles/valu_mix.json) per config,
#       then tools/replay_count.sh for C2's helper-wave layout (unless NO_REPLAY=1; needs
#       build/abl/libmbik_replay.so)
#   tools/evidence.sh kstats             TAG, KSTATS="name:bench args;..."
#       rocprofv3 --kernel-trace --stats of pinned layouts                 -> gpurun_out/$TAG/<name>/
#   tools/evidence.sh profile <tag> <cfg>
#       tools/round_profile.sh (bench line, kernel stats, keyed PMC traffic), then the VALU mix
#       of the layout that pass timed
set -o pipefail
cd "$(dirname "$0")/.."
ROOT=$PWD
CMD=${1:-call}
shift || true
TAG=${TAG:-r05}
OUT=$ROOT/gpurun_out/$TAG

suite() {
  mkdir -p $OUT
  timeout -k 10 ${SUITE_S:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gpu_suite.log 2>&1
  local rc=$?; echo "suite rc=$rc $(date +%T)"; tail -3 $OUT/gpu_suite.log; return $rc
}
smoke() {
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  local rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; return $rc
}
bench() { # <output name> <bench.py args...>
  local name=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?; echo "bench[$*] rc=$rc"; tail -c 500 $OUT/$name.json; echo; return $rc
}

case $CMD in
call)
  echo "start $(date +%T)"
  suite || exit 1
  if [ -n "$SMOKE" ]; then smoke || exit 1; fi
  if [ -n "$BENCH" ]; then
    i=0
    IFS=';' read -ra BS <<< "$BENCH"
    for b in "${BS[@]}"; do bench bench_$i $b || exit 1; i=$((i+1)); done
  fi
  echo "done $(date +%T)";;
final)
  echo "start $(date +%T)"
  suite || exit 1
  smoke || exit 1
  bench c2_bench || exit 1
  mkdir -p $OUT/prof
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 $ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2_prof_bench.json 2> $OUT/c2_prof.err) || { echo "rocprof failed"; exit 1; }
  for c in 3 4 5; do bench c${c}_bench --config $c --steps 10 --warmup 2 || exit 1; done
  for c in 5 2; do bench c${c}_cmode_bench --config $c --constraint-mode --steps 10 --warmup 3 || exit 1; done
  echo "done $(date +%T)";;
counters)
  declare -A LAY=([2]="4:16:1:1:0:1:1" [3]="4:16:4:4:1:2:0" [4]="4:16:1:4:2:2:0" [5]="8:8:1:4:2:2:0")
  for kv in $LAYOUTS; do LAY[${kv%%:*}]=${kv#*:}; done
  echo "start $(date +%T)"
  for c in ${CFGS:-2 3 4 5}; do
    O=$OUT/c$c
    mkdir -p $O
    for ctr in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && TMPDIR=/tmp timeout -s KILL 240 rocprofv3 --pmc $ctr -d $O/$ctr -o run --output-format csv -- \
        python3 $ROOT/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-parity --layout ${LAY[$c]} \
        > $O/$ctr.json 2> $O/$ctr.log) || { echo "c$c $ctr pass failed"; tail -5 $O/$ctr.log; exit 1; }
    done
    bash tools/valu_mix.sh $TAG/mix_c$c $c ${LAY[$c]} > $O/mix.log 2>&1 || { echo "c$c mix passes failed"; tail -5 $O/mix.log; exit 1; }
    echo "c$c done $(date +%T)"
  done
  if [ -z "$NO_REPLAY" ]; then
    bash tools/replay_count.sh $TAG/replay 2:4096 > $OUT/replay.log 2>&1 || { echo "replay failed"; tail -5 $OUT/replay.log; exit 1; }
    head -2 $OUT/replay.log
  fi
  echo "done $(date +%T)";;
kstats)
  # rocprofv3 kernel stats of pinned layouts (no autotune launches in the averages):
  # KSTATS="name:bench args;..." (default: the round's C4 / C5 / C5 constraint_mode picks)
  KS=${KSTATS:-"c4:--config 4 --layout 4:64:1:0:2:2:0:1;c5:--config 5 --layout 8:64:2:0:2:2:0:1;c5cm:--config 5 --constraint-mode --layout 8:64:1:1:0:1:0:1"}
  mkdir -p $OUT
  IFS=';' read -ra KA <<< "$KS"
  for kv in "${KA[@]}"; do
    n=${kv%%:*}; args=${kv#*:}
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run --output-format csv -- \
      python3 $ROOT/bench.py $args --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$n.json 2> $OUT/$n.err) || { echo "$n failed"; exit 1; }
    echo "$n done"
  done;;
profile)
  T=$1; CFG=$2
  bash tools/round_profile.sh $T $CFG || exit 1
  bash tools/valu_mix.sh ${T}_mix $CFG $(python3 tools/layout_of.py gpurun_out/$T/bench.json);;
*)
  echo "usage: tools/evidence.sh call|final|counters|kstats|profile ..." >&2; exit 2;;
esac
