#!/bin/bash
# Dynamic VALU instruction mix of the solve kernel (SQ_INSTS_VALU_* classes, one rocprofv3
# --pmc pass per group of <= 8 SQ counters), summed over the kernel's dispatches:
#   tools/valu_mix.sh <tag> [config] [layout K:spw:interval:staging:placement:waves]
#     ->  gpurun_out/<tag>/g*/run_counter_collection.csv, gpurun_out/<tag>/mix.json
# With a layout the passes time exactly that layout (bench.py --layout); without one, the
# default layout (--no-autotune).  tools/mix_entry.py turns mix.json into a valu_mix.json entry.
set -e
TAG=${1:-mix}; CFG=${2:-2}; LAYOUT=${3:-}
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-parity"
if [ -n "$LAYOUT" ]; then B="$B --layout $LAYOUT"; else B="$B --no-autotune"; fi
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32" \
         "SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU SQ_WAVE_CYCLES" \
         "SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VSKIPPED"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G -d $OUT/g$i -o run --output-format csv -- python3 $B > $OUT/g$i.json 2> $OUT/g$i.log
done
python3 $ROOT/tools/pmc_sum.py $OUT/g*/run_counter_collection.csv > $OUT/mix.json
cat $OUT/mix.json
