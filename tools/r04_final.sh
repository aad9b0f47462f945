#!/bin/bash
# Round-4 evidence in one gpurun call: the whole -m gpu suite, smoke(), the default bench line
# (C2), its rocprofv3 kernel stats, the C3/C4/C5 bench lines, each step under its own limit.
set -o pipefail
TAG=${TAG:-r04z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "start $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "suite failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/c2_bench.json 2> $OUT/c2_bench.err || { echo "bench failed"; tail $OUT/c2_bench.err; exit 1; }
tail -c 400 $OUT/c2_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/c2_prof_bench.json 2> $GRAFT_REPO_ROOT/$OUT/c2_prof.err || { echo "rocprof failed"; exit 1; }
cd $GRAFT_REPO_ROOT
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 2 > $OUT/c${c}_bench.json 2> $OUT/c${c}_bench.err || { echo "bench c$c failed"; exit 1; }
done
echo "done $(date +%T)"
