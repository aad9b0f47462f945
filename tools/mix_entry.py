"""Turn one tools/valu_mix.sh run into a profiles/valu_mix.json entry, keyed like traffic.json
(config, size and the layout the passes timed, from their bench lines' roofline.traffic_key):
    python tools/mix_entry.py <gpurun_out/tag> [profiles/valu_mix.json]"""
import json
import os
import sys

src = sys.argv[1]
dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "valu_mix.json")
keys = set()
for g in ("g1", "g2", "g3"):
    line = open(os.path.join(src, g + ".json")).read().strip().splitlines()[-1]
    keys.add(json.loads(line)["roofline"]["traffic_key"])
if len(keys) != 1:
    sys.exit(f"the passes timed different layouts: {sorted(keys)}")
key = keys.pop()
m = json.load(open(os.path.join(src, "mix.json")))
classes = {k[len("SQ_INSTS_VALU_"):]: m[k] for k in m if k.startswith("SQ_INSTS_VALU_") and k != "SQ_INSTS_VALU_"}
valu = m["SQ_INSTS_VALU"]
classes["OTHER_mov_cmp_cndmask_bitwise"] = valu - sum(classes.values())
wave_cycles = 4 * m["SQ_WAVE_CYCLES"]
entry = {
    "source": f"tools/valu_mix.sh (3 rocprofv3 --pmc passes of bench.py, layout {key}), per wave, mean over the "
              "solve dispatches; SQ_WAVE_CYCLES is in 4-cycle units"
              + ("; helper-wave layout: two waves per block (the solving wave and its helper), so every per-wave "
                 "value is the mean of the two" if key.endswith("_h1") else ""),
    "valu_insts_per_wave": valu,
    "wave_cycles": wave_cycles,
    "valu_issue_floor_cycles": 4 * valu,
    "issue_frac": 4 * valu / wave_cycles,
    "valu_classes_per_wave": dict(sorted(classes.items())),
    "salu_insts_per_wave": m.get("SQ_INSTS_SALU"),
    "lds_insts_per_wave": m.get("SQ_INSTS_LDS"),
    "vmem_insts_per_wave": m.get("SQ_INSTS_VMEM"),
    "branch_insts_per_wave": m.get("SQ_INSTS_BRANCH"),
}
vm = json.load(open(dst)) if os.path.exists(dst) else {}
vm[key] = entry
json.dump(vm, open(dst, "w"), indent=1, sort_keys=True)
print(key, json.dumps(entry))
