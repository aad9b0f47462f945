"""Solving-wave VALU accounting of a helper-wave launch from the two
rocprofv3 --pmc passes of tools/replay_count.sh:
  * the helper-wave launches (mbik_solve_kernel_help, two waves per block): wave cycles (both
    waves live for the whole launch, so the per-wave mean is the solving wave's lifetime) and
    the block's total VALU;
  * the replay launch (mbik_solve_kernel_replay: the solving wave alone, reading the saved
    helper records; bitwise equal output): the solving wave's own VALU instructions.
Solving-wave issue fraction = 4 cycles x its VALU instructions / its wave cycles (one wave
issues at most one VALU instruction per 4 cycles, MI355X_MICROARCH).  The helper's share is the
block total minus the solving wave's (its spin polls included).
    python tools/solver_issue.py gpurun_out/<tag> <valu_mix key>   -> merged into profiles/valu_mix.json"""
import collections
import csv
import json
import os
import sys

tag_dir, key = sys.argv[1], sys.argv[2]
per = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for g in ("g1", "g2"):
    path = os.path.join(tag_dir, g, "run_counter_collection.csv")
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        kind = "help" if "solve_kernel_help" in k else ("replay" if "solve_kernel_replay" in k else None)
        if kind:
            disp[(kind, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (kind, d), c in disp.items():
        for name, v in c.items():
            per[(g, kind)][name] += v
        n[(g, kind)] += 1
mean = {gk: {name: v / n[gk] for name, v in c.items()} for gk, c in per.items()}
h1, r1 = mean[("g1", "help")], mean[("g1", "replay")]
h2, r2 = mean[("g2", "help")], mean[("g2", "replay")]
blocks = r1["SQ_WAVES"]                                   # one solving wave per block
wave_cycles = 4.0 * h1["SQ_WAVE_CYCLES"] / h1["SQ_WAVES"]  # quad-cycles -> cycles, mean of the two waves
solver_valu = r1["SQ_INSTS_VALU"] / blocks
block_valu = h1["SQ_INSTS_VALU"] / blocks
out = {
    "solver_valu_insts_per_wave": round(solver_valu, 1),
    "solver_wave_cycles": round(wave_cycles, 1),
    "solver_issue_frac": 4.0 * solver_valu / wave_cycles,
    "solver_valu_issue_floor_cycles": round(4.0 * solver_valu, 1),
    "helper_valu_insts_per_wave": round(block_valu - solver_valu, 1),
    "helper_issue_frac": 4.0 * (block_valu - solver_valu) / wave_cycles,
    "solver_lds_insts_per_wave": round(r1["SQ_INSTS_LDS"] / blocks, 1),
    "solver_salu_insts_per_wave": round(r1["SQ_INSTS_SALU"] / blocks, 1),
    "solver_valu_classes_per_wave": {name[len("SQ_INSTS_VALU_"):]: round(r2[name] / r2["SQ_WAVES"], 1)
                                     for name in r2 if name.startswith("SQ_INSTS_VALU_")},
    "replay_wave_cycles": round(4.0 * r1["SQ_WAVE_CYCLES"] / r1["SQ_WAVES"], 1),
    "solver_source": "tools/replay_count.sh + tools/solver_issue.py: VALU of the solving wave alone (mbik_solve_kernel_replay, "
                     "the saved helper records, bitwise-equal output) over the wave cycles of the helper-wave launch",
}
vm_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "valu_mix.json")
vm = json.load(open(vm_path))
vm.setdefault(key, {}).update(out)
json.dump(vm, open(vm_path, "w"), indent=1, sort_keys=True)
print(json.dumps(out, indent=1))
