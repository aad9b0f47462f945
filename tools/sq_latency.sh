#!/bin/bash
# PMC latency/level counters (LDS, VMEM, SMEM) of the solve kernel: CFG=<cfg> tools/sq_latency.sh
set -e
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/sqlat
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --config ${CFG:-2} --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-autotune"
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES -d $OUT/g1 -o run --output-format csv -- python3 $B > $OUT/g1.json 2> $OUT/g1.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM_NORM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $OUT/g2 -o run --output-format csv -- python3 $B > $OUT/g2.json 2> $OUT/g2.log
