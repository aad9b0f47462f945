#!/bin/bash
# SQ instruction / cycle counters of the solve kernel (one rocprofv3 --pmc pass per group).
#   tools/sq_counters.sh <tag> [config] [extra bench args]
set -e
TAG=${1:-sq}; CFG=${2:-2}; shift 2 || true
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-parity --no-autotune $*"
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $G -d $OUT/g$i -o run --output-format csv -- python3 $B > $OUT/g$i.json 2> $OUT/g$i.log
done
