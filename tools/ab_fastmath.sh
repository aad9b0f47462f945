set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
for tag in NEW IEEE; do
  if [ $tag = NEW ]; then unset MBIK_LIB_OVERRIDE; else export MBIK_LIB_OVERRIDE=$PWD/build/abl/libmbik_abl_$tag.so; fi
  echo "== $tag"; timeout -k 10 200 python tools/sweep.py 2:4096:4 3:65536:4 5:16384:16 2>/dev/null
done
