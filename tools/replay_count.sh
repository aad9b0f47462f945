#!/bin/bash
# Solving-wave VALU accounting of helper-wave launches (tools/replay_count.py): builds the
# -DMBIK_REPLAY library, runs the replay once plainly (timing + bitwise check), then one
# rocprofv3 --pmc pass per counter group.  -> gpurun_out/<tag>/
#   tools/replay_count.sh <tag> CFG:N [...]      (run on the GPU box)
set -e
TAG=${1:-replay}; shift
CASES=${@:-2:4096}
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export MBIK_LIB_OVERRIDE=${REPLAY_LIB:-$ROOT/build/diag/libmbik_replay.so}  # (OUT=build/diag/libmbik_replay.so tools/prof_build.sh REPLAY)
timeout -k 10 120 python3 -u tools/replay_count.py $CASES > $OUT/plain.jsonl 2> $OUT/plain.err
cat $OUT/plain.jsonl
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G -d $OUT/g$i -o run --output-format csv -- python3 $ROOT/tools/replay_count.py $CASES > $OUT/g$i.jsonl 2> $OUT/g$i.log
done
ls $OUT/g*/
