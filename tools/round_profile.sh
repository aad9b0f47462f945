#!/bin/bash
# One GPU-box pass for the round's evidence: bench line, kernel-trace stats, PMC traffic.
#   tools/round_profile.sh <round-tag> [config]
# Every GPU step has its own time limit; the first failure ends the script.
set -e
TAG=${1:-r01}; CFG=${2:-2}
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="$ROOT/bench.py --config $CFG --steps 20 --warmup 3 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run --output-format csv -- python3 $B > $OUT/ktrace.json 2> $OUT/ktrace.log
# the PMC passes and the final bench line run the layout the kernel-trace run's autotune picked
LAYOUT=$(python3 -c "import json; c=json.loads(open('$OUT/ktrace.json').read().strip().splitlines()[-1])['config']; l=c['layout']; print(':'.join(str(x) for x in (c['lanes_per_skeleton'], c['skeletons_per_block'], l['checkpoint_interval'], l['heading_staging'], l['state_placement'], l['waves_per_simd'], l.get('helper_wave', 0))))")
B="$B --layout $LAYOUT"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B > $OUT/fetch.json 2> $OUT/fetch.log
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B > $OUT/write.json 2> $OUT/write.log
# keyed by config, size and the layout the PMC runs' autotune picked (bench.py reads the key of
# the layout it times); a pass whose layout differs from the kernel-trace run's is reported
KEY=$(python3 -c "import json; d=json.loads(open('$OUT/fetch.json').read().strip().splitlines()[-1]); print(d['roofline']['traffic_key'])")
KEYW=$(python3 -c "import json; d=json.loads(open('$OUT/write.json').read().strip().splitlines()[-1]); print(d['roofline']['traffic_key'])")
[ "$KEY" = "$KEYW" ] || { echo "FETCH and WRITE passes picked different layouts: $KEY vs $KEYW"; exit 3; }
# the last 26 dispatches: 20 timed steps + 6 host-buffer frames, after autotune fixed the layout
python3 tools/traffic_from_pmc.py $(ls $OUT/fetch/run_counter_collection.csv) $(ls $OUT/write/run_counter_collection.csv) $KEY profiles/traffic.json --last 26
cp profiles/traffic.json $OUT/traffic.json
timeout -k 10 300 python3 bench.py --config $CFG --layout $LAYOUT > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
