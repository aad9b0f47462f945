#!/bin/bash
# Round-3 diagnostic call (one gpurun): the placement-2 state-in-device-memory parity cases under
# the diagnostic builds of build/diag (MBIK_CHECK_BOUNDS, and the SGPR-offset variants of
# DESIGN.md §10), with -s so device printf reaches the log.
# Stops at the first step that ends in anything but pass (0) or test failures (1).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03diag
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for v in ${@:-chk soff_chk soff soff_sync soff_rfl soff_tgst soff_hs soff_nohs}; do
  MBIK_LIB_OVERRIDE=build/diag/libmbik_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_layouts.py -m gpu -q -s \
    -k "test_state_in_hbm_bitwise_vs_oracle" --timeout 240 --timeout-method thread > gpurun_out/r03diag/layouts_$v.log 2>&1
  rc=$?; echo "$v rc=$rc oob=$(grep -c 'mbik OOB' gpurun_out/r03diag/layouts_$v.log)"; tail -1 gpurun_out/r03diag/layouts_$v.log; ok $rc || exit $rc
done
