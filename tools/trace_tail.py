"""Average mbik_solve_kernel duration over the last N dispatches of a rocprofv3 kernel trace
(bench.py's timed steps come after mbik_plan_autotune's candidate launches, which the
--stats summary averages in):  python tools/trace_tail.py <run_kernel_trace.csv> [N=26]"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mbik_solve_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 26
tail = rows[-n:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tail]
print(json.dumps({"dispatches": len(d), "avg_ms": sum(d) / len(d), "min_ms": min(d), "max_ms": max(d), "all_dispatches": len(rows)}))
