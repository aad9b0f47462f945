#!/bin/bash
# A config's whole evidence pass: tools/round_profile.sh (bench line, kernel stats, keyed PMC
# traffic), then tools/valu_mix.sh on the layout that pass timed.
#   tools/evidence.sh <tag> <config>
set -e
TAG=$1; CFG=$2
cd "$(dirname "$0")/.."
bash tools/round_profile.sh $TAG $CFG
bash tools/valu_mix.sh ${TAG}_mix $CFG $(python3 tools/layout_of.py gpurun_out/$TAG/bench.json)
