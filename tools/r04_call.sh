#!/bin/bash
# One gpurun call of round 4: selected -m gpu tests (TESTS, default the whole suite), then
# optionally smoke() and a bench line (BENCH="--config 2 ..."), each under its own time limit;
# stops at the first step that ends badly.
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-r04}
mkdir -p $OUT
echo "start $(date +%T)"
timeout -k 10 ${SUITE_S:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc $(date +%T)"; tail -5 $OUT/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH" ]; then
  i=0
  IFS=';' read -ra BS <<< "$BENCH"
  for b in "${BS[@]}"; do
    timeout -k 10 400 python -u bench.py $b > $OUT/bench_$i.json 2> $OUT/bench_$i.err
    rc=$?; echo "bench[$b] rc=$rc"; tail -c 600 $OUT/bench_$i.json; [ $rc -eq 0 ] || exit $rc
    i=$((i+1))
  done
fi
echo "done $(date +%T)"
