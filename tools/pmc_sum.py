"""Sum rocprofv3 counter_collection.csv files per counter over the solve kernel's dispatches
and print per-wave values (counter / SQ_WAVES) as JSON."""
import csv
import json
import sys
from collections import defaultdict

tot = defaultdict(float)
for path in sys.argv[1:]:
    waves = defaultdict(float)
    vals = defaultdict(float)
    for row in csv.DictReader(open(path)):
        if "mbik_solve_kernel" not in row.get("Kernel_Name", ""):
            continue
        name, v = row["Counter_Name"], float(row["Counter_Value"])
        (waves if name == "SQ_WAVES" else vals)[name] += v
    w = sum(waves.values())
    for k, v in vals.items():
        tot[k] = v / w if w else float("nan")
    tot["SQ_WAVES_per_dispatch_total"] = w
print(json.dumps({k: round(v, 1) for k, v in sorted(tot.items())}, indent=1))
