#!/bin/bash
# Instruction-cache counters of the solve kernel: tools/icache_counters.sh <tag> <config> [bench args]
set -e
TAG=${1:-ic}; CFG=${2:-2}; shift 2 || true
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-autotune $*"
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d $OUT/ic -o run --output-format csv -- python3 $B > $OUT/ic.json 2> $OUT/ic.log
