"""Copy one tools/round_profile.sh run into profiles/: kernel stats, the post-autotune trace
average, PMC passes, the bench line (its traffic and kernel average taken over the same
post-autotune dispatches) and the traffic.json entry.
    python tools/evidence_to_profiles.py <gpurun_out/tag> <config> [round=r01]"""
import json
import os
import shutil
import subprocess
import sys

src, cfg = sys.argv[1], int(sys.argv[2])
rnd = sys.argv[3] if len(sys.argv) > 3 else "r02"
here = os.path.dirname(os.path.abspath(__file__))
prof = os.path.join(here, "..", "profiles")
c = f"c{cfg}"
shutil.copy(f"{src}/ktrace/run_kernel_stats.csv", f"{prof}/{rnd}_{c}_kernel_stats.csv")
tail = subprocess.run([sys.executable, f"{here}/trace_tail.py", f"{src}/ktrace/run_kernel_trace.csv", "26"],
                      check=True, capture_output=True, text=True).stdout
open(f"{prof}/{rnd}_{c}_trace_tail.json", "w").write(tail)
shutil.copy(f"{src}/fetch/run_counter_collection.csv", f"{prof}/{rnd}_{c}_pmc_fetch_size.csv")
shutil.copy(f"{src}/write/run_counter_collection.csv", f"{prof}/{rnd}_{c}_pmc_write_size.csv")
bench = json.loads(open(f"{src}/bench.json").read().strip().splitlines()[-1])
t = json.load(open(f"{src}/traffic.json"))
key = bench["roofline"]["traffic_key"]     # config, size and the layout timed
tj_path = f"{prof}/traffic.json"
tj = json.load(open(tj_path))
tj[key] = t[key]
json.dump(tj, open(tj_path, "w"), indent=1, sort_keys=True)
vm = json.load(open(f"{prof}/valu_mix.json")).get(key)
# the instruction-mix pass of this layout (tools/mix_entry.py), as bench.py reports it
bench["issue"] = None if not vm else {
    "bound": "valu_issue_1wave", "achieved_cycles_per_wave": vm["valu_issue_floor_cycles"],
    "wave_cycles": vm["wave_cycles"], "frac": vm["issue_frac"],
    "note": "4 cycles per wave64 VALU instruction x VALU instructions / wave cycles (PMC, "
            "profiles/valu_mix.json); the ceiling this latency-bound chain runs against"}
json.dump(bench, open(f"{prof}/{rnd}_{c}_bench.json", "w"))
print(key, bench["ms_per_step"], bench["value"], bench["config"].get("layout"), json.loads(tail)["avg_ms"])
