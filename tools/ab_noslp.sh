set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
for tag in BASE NOSLP; do
  export MBIK_LIB_OVERRIDE=$PWD/build/abl/libmbik_abl_$tag.so
  echo "== $tag"
  timeout -k 10 200 python tools/sweep.py 5:16384:16 2>/dev/null || exit 1
  timeout -k 10 200 python bench.py --config 2 --constraint-mode --no-cpu-baseline --no-parity 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('cmode c2', d['ms_per_step'])" || exit 1
  timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --no-parity 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c3 autotuned', d['ms_per_step'])" || exit 1
done
