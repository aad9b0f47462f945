"""Heterogeneous crowd: several rigs solved per frame by one mbik_group_solve launch vs one
mbik_solve launch per rig on the same stream (same results; prints ms per frame)."""
import json
import sys

import torch

sys.path.insert(0, '.')
from many_bone_ik_amd import workloads as W
from many_bone_ik_amd.solver import Group, Plan

dev = torch.device('cuda', 0)
crowd = [(2, 1024), (5, 256), (3, 4096), (4, 2048)]
if len(sys.argv) > 1:
    crowd = [tuple(int(x) for x in c.split(':')) for c in sys.argv[1:]]
plans, bufs = [], []
for cfg, n in crowd:
    wl = W.generate(cfg, n)
    plans.append(Plan.from_workload(wl))
    pi = torch.from_numpy(wl.pose).to(dev)
    tg = torch.from_numpy(wl.targets).to(dev)
    bufs.append((pi, tg, torch.empty_like(pi), torch.empty_like(pi)))
st = torch.cuda.current_stream(dev).cuda_stream
g = Group(plans)


def fused():
    g.solve([b[0].data_ptr() for b in bufs], [b[1].data_ptr() for b in bufs], [b[2].data_ptr() for b in bufs], stream=st)


def separate():
    for p, b in zip(plans, bufs):
        p.solve(b[0].data_ptr(), b[1].data_ptr(), b[3].data_ptr(), 0, p.n, st)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ms_sep = timed(separate)
ms_fused = timed(fused)
same = all(torch.equal(b[2], b[3]) for b in bufs)
total = sum(n for _, n in crowd)
print(json.dumps(dict(crowd=[f"C{c} x {n}" for c, n in crowd], skeletons=total, ms_separate=round(ms_sep, 3),
                      ms_group=round(ms_fused, 3), speedup=round(ms_sep / ms_fused, 3),
                      group_skeletons_per_s=round(total / ms_fused * 1e3), bitwise_equal=same)))
