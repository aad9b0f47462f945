#!/bin/bash
# One gpurun call: diagnostics (tools/r03_diag.sh), the -m gpu suite, then an A/B of
# build/abl variants (tools/variant_check.py).  Stops at the first step that ends badly.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r03
if [ -n "$DIAG" ]; then bash tools/r03_diag.sh $DIAG || exit $?; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r03/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$AB" ]; then
  timeout -k 10 900 python -u tools/variant_check.py --reps 2 --cases ${CASES:-2:4096,4:32768,5:16384} $AB > gpurun_out/r03/ab.jsonl 2> gpurun_out/r03/ab.err
  rc=$?; echo "ab rc=$rc"; cat gpurun_out/r03/ab.jsonl; exit $rc
fi
