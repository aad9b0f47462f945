#!/bin/bash
# Where a solve wave's cycles go (MI355X_MICROARCH counter table: SQ_WAIT_ANY = parked at
# s_waitcnt / barrier / sleep, SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_ANY = issuing;
# the three add up to SQ_WAVE_CYCLES), plus L2 hit rate, per config:
#   tools/stall_counters.sh <tag> 2:LAYOUT 4:LAYOUT ...    -> gpurun_out/<tag>/s<spec#>_c<cfg>_g<i>/
# LAYOUT "auto": the bench's autotuned layout; EXTRA: more bench.py arguments (--constraint-mode);
# TRAFFIC=1 adds FETCH_SIZE and WRITE_SIZE passes (groups 4 and 5)
set -e
TAG=${1:-stall}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
n=0
for spec in "$@"; do
  n=$((n+1))
  CFG=${spec%%:*}; LAYOUT=${spec#*:}
  LA="--layout $LAYOUT"; [ "$LAYOUT" = auto ] && LA=
  B="$ROOT/bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-parity $LA $EXTRA"
  i=0
  for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_VALU" \
           "SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum" ${TRAFFIC:+FETCH_SIZE WRITE_SIZE}; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G -d $OUT/s${n}_c${CFG}_g$i -o run --output-format csv -- python3 $B > $OUT/s${n}_c${CFG}_g$i.json 2> $OUT/s${n}_c${CFG}_g$i.log
  done
done
ls $OUT
