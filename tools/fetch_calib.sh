#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes of tools/fetch_calib.hip (one PMC pass each).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/fc
timeout -k 10 120 build/fetch_calib > gpurun_out/fc/times.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/fc/fetch -o fc --output-format csv -- build/fetch_calib > gpurun_out/fc/pmc.log 2>&1 || exit $?
cat gpurun_out/fc/times.txt
