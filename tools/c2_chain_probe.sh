#!/bin/bash
# C2's solving-wave chain: load-site ablations (SOA = setup tables, MEM = every load site) on the
# shipped helper-wave layout, interleaved, and the phase split of the same layout (MBIK_PROF).
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-c2chain}; O=gpurun_out/$TAG; mkdir -p $O
TAG=$TAG REPS=3 STEPS=20 timeout -k 10 500 bash tools/ab_env.sh "base||build/diag/libmbik_abl_BASE.so" \
  "SOA||build/diag/libmbik_abl_SOA.so" "MEM||build/diag/libmbik_abl_MEM.so" -- 2:4:16:1:1:0:1:1:0 > $O/ab.log 2>&1 || { echo ab failed; tail -5 $O/ab.log; exit 1; }
cat $O/ab.log
MBIK_HELP=1 MBIK_LIB_OVERRIDE=$PWD/build/diag/libmbik_abl_PROF.so timeout -k 10 200 python tools/prof_phases.py 2:4096:4:16:1:1:0:1 \
  > $O/phases.jsonl 2> $O/phases.err || { echo phases failed; tail -5 $O/phases.err; exit 1; }
cat $O/phases.jsonl
