#!/bin/bash
export MBIK_BENCH_PMC=${MBIK_BENCH_PMC:-off}  # timing-only bench runs: no live counter leg
# what do the helper-wave kernel's SGPR spills cost C2?  27 of the SGPRs it
# keeps live are the topology tables' LDS offsets.  A timing-only build with the C2 plan's offsets
# compiled in (tools/topo_const.py, solve_block.h MBIK_TOPO_CONST) frees them; same-box A/B of
# that build against the in-tree library on C2's bench layout (the bench's parity check confirms
# the constant offsets are the timed plan's).           TAG=r06d tools/c2_topo_const_ab.sh
set -o pipefail
cd "$(dirname "$0")/.."
TAG=${TAG:-tconst}
OUT=gpurun_out/$TAG
mkdir -p $OUT
LAYOUT=${LAYOUT:-4:16:1:1:0:1:1:0}
timeout -k 10 300 python tools/topo_const.py 2 4096 $LAYOUT || exit 1
cp build/diag/topo_const.h $OUT/
timeout -k 10 900 python -m many_bone_ik_amd.build --variant build/diag/libmbik_abl_TCONST.so -DMBIK_TOPO_CONST -I$PWD/build/diag \
  > $OUT/build.log 2>&1 || { echo build failed; tail -20 $OUT/build.log; exit 1; }
TAG=$TAG REPS=${REPS:-3} timeout -k 10 600 bash tools/ab_env.sh "base||-" "tconst||build/diag/libmbik_abl_TCONST.so" -- 2:$LAYOUT
