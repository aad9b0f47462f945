#!/bin/bash
# Round-6 pass: C4 strong line on the wave-roles layout (262,144 skeletons, pinned: autotune at
# that size runs minutes), C3 pinned to the wave-roles layout, and the N = 2 rehearsal on one
# GPU (gloo, library_multi on 0,0).
set -o pipefail
O=gpurun_out/${TAG:-r06i}; mkdir -p $O
echo "strong $(date +%T)"
timeout -k 10 500 python -u bench.py --config 4 --scaling strong --layout 4:64:1:0:2:2:0:1 --steps 5 --warmup 2 --no-cpu-baseline --pmc off \
  > $O/c4_strong.json 2> $O/c4_strong.err || { echo strong failed; tail -5 $O/c4_strong.err; exit 1; }
echo "c3 wave roles $(date +%T)"
timeout -k 10 300 python -u bench.py --config 3 --layout 4:64:1:0:2:2:0:1 --steps 10 --warmup 2 --no-cpu-baseline \
  > $O/c3_rw.json 2> $O/c3_rw.err || { echo c3 rw failed; tail -5 $O/c3_rw.err; exit 1; }
echo "rehearsal $(date +%T)"
MBIK_BENCH_DEVICE=0 MBIK_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --library-multi-devices 0,0 \
  > $O/n2_rehearsal.json 2> $O/n2_rehearsal.err || { echo rehearsal failed; tail -5 $O/n2_rehearsal.err; exit 1; }
echo "done $(date +%T)"
