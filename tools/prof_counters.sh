#!/bin/bash
# PMC passes for one bench config (each counter group in its own rocprofv3 run).
set -e
CFG=${1:-2}; TAG=${2:-c$CFG}
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
run() { timeout -k 10 240 rocprofv3 --pmc $1 -d $OUT/$2 -o run --output-format csv -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/$2.log 2>&1; }
run "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" p1
run "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" p2
run "FETCH_SIZE" p3
run "WRITE_SIZE" p4
