"""Print the bench --layout argument (K:spw:interval:staging:placement:waves:helper) of a bench.py JSON
line file:  python tools/layout_of.py gpurun_out/<tag>/bench.json"""
import json
import sys

c = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["config"]
l = c["layout"]
print(":".join(str(x) for x in (c["lanes_per_skeleton"], c["skeletons_per_block"], l["checkpoint_interval"],
                                l["heading_staging"], l["state_placement"], l["waves_per_simd"], l.get("helper_wave", 0))))
