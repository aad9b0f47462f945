"""Summarise tools/stall_counters.sh output: per config, the solve kernel's counters averaged over
its dispatches, per wave (SQ_*: quad-cycles -> cycles), and the L2 hit rate.
    python tools/stall_summary.py gpurun_out/<tag>"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
out = {}
for g in sorted(glob.glob(os.path.join(d, "c*_g*"))):
    if not os.path.isdir(g):
        continue
    cfg = os.path.basename(g).split("_")[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for path in glob.glob(os.path.join(g, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "solve_kernel" not in r["Kernel_Name"]:
                continue
            acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    disp = list(acc.values())[-4:]  # after autotune / warmup: the timed layout's launches
    if not disp:
        continue
    mean = {k: sum(x.get(k, 0.0) for x in disp) / len(disp) for k in disp[0]}
    out.setdefault(cfg, {}).update(mean)
res = {}
for cfg, m in out.items():
    w = m.get("SQ_WAVES", 1.0)
    r = {"waves": w}
    for k, v in m.items():
        if k.startswith("SQ_") and k != "SQ_WAVES":
            r[k] = v / w * (4 if ("CYCLES" in k or "WAIT" in k or "ACTIVE" in k) else 1)
    if "SQ_WAVE_CYCLES" in m:
        wc = r["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
            if k in r:
                r[k + "_frac"] = r[k] / wc
    if "TCC_HIT_sum" in m:
        r["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
        r["tcc_requests"] = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
    res[cfg] = {k: round(v, 4) if isinstance(v, float) else v for k, v in r.items()}
print(json.dumps(res, indent=1))
